"""Model-level parity: the plugins (through libvspike) vs golden fixtures generated from the
reference (oracle/gen_fixtures.py) and vs the CPU restatement (oracle/cpu_ref.py).

Tolerances (north star: outputs within 1e-4 relative in fp32, loss curve within 1e-3):
  * fp32 mode: log-rates / hidden states 1e-4 relative to max|ref|; grads 1e-3 of the tensor norm
    (norm-relative, see cpu_ref.compare_summary); loss curves 1e-3 relative.
  * bf16 mode: log-rates 3e-2 relative to max|ref|, loss 1e-2 relative (bf16 activations).
"""
import numpy as np
import pytest
import torch

from oracle import cpu_ref, prng

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _vit_model(cfg: cpu_ref.ViTCfg, enc_out, n, dtype="fp32", freeze=False):
    from vspike import VideoMAE
    conf = {"model_class": "VideoMAE", "freeze_encoder": freeze, "compute_dtype": dtype,
            "backbone": {k: getattr(cfg, k) for k in ("image_size", "patch_size", "num_channels", "num_frames",
                                                       "tubelet_size", "hidden_size", "num_hidden_layers",
                                                       "num_attention_heads", "intermediate_size",
                                                       "layer_norm_eps")},
            "encoder": {"output_dim": enc_out}, "decoder": {"output_dim": 100 * n}}
    m = VideoMAE(conf).to(DEV)
    m.load_reference_state_dict({k: torch.from_numpy(v) for k, v in cpu_ref.make_vit_params(cfg, enc_out, n).items()})
    return m


def _maxrel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def test_vit_small_fp32_forward_backward_matches_reference(golden):
    from vspike import poisson_nll_mean
    from vspike.layout import modern_name
    fx = golden("vit_small.npz")
    cfg, B, n = cpu_ref.VIT_SMALL_FIXTURE, 2, 16
    m = _vit_model(cfg, 64, n)
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B)).to(DEV)
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n))).to(DEV)
    out = m(px)
    assert _maxrel(out.detach().cpu(), fx["log_rates"]) < 1e-4
    loss = poisson_nll_mean(out, y)
    assert abs(loss.item() - fx["loss"][0]) < 1e-5 * abs(fx["loss"][0])
    loss.backward()
    sd = {}
    # map flat grads back to reference names
    for name, which, slot, rows in m.layout.hf_items():
        flat = m.enc_flat.grad if which == "enc" else m.head_flat.grad
        t = (m.layout.enc if which == "enc" else m.layout.head).view(flat, slot)
        sd[modern_name(name)] = (t if rows is None else t[rows]).detach().cpu().numpy()
    for name, g in sd.items():
        shape = cpu_ref.vit_param_shapes(cfg, 64, n)[name]
        ok, msg = cpu_ref.compare_summary(name, g.reshape(shape), fx, rtol=1e-3, atol=1e-8)
        assert ok, msg


def test_vit_small_bf16_close_to_reference(golden):
    fx = golden("vit_small.npz")
    cfg, B, n = cpu_ref.VIT_SMALL_FIXTURE, 2, 16
    m = _vit_model(cfg, 64, n, dtype="bf16")
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B)).to(DEV)
    out = m(px)
    assert _maxrel(out.detach().cpu(), fx["log_rates"]) < 3e-2


def test_vit_tiny_full_tokens_fp32(golden):
    fx = golden("vit_tiny1l.npz")
    cfg = cpu_ref.ViTCfg(hidden_size=192, num_attention_heads=3, intermediate_size=768, num_hidden_layers=1)
    m = _vit_model(cfg, 64, 8, freeze=True)
    with torch.no_grad():
        out = m(torch.from_numpy(cpu_ref.make_pixels(cfg, 1)).to(DEV))
    assert _maxrel(out.cpu(), fx["log_rates"]) < 1e-4


@pytest.mark.parametrize("frozen", [True, False])
def test_vit_small_loss_curve_matches_reference(golden, frozen):
    from vspike import FusedAdamW, poisson_nll_mean
    fx = golden("vit_small.npz")
    cfg, B, n = cpu_ref.VIT_SMALL_FIXTURE, 2, 16
    m = _vit_model(cfg, 64, n, freeze=frozen)
    opt = FusedAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-5, weight_decay=0.01, eps=1e-8)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, total_steps=4, max_lr=1e-5, pct_start=0.15, div_factor=10)
    losses = []
    for s in range(4):
        px = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=300 + s)).to(DEV)
        y = torch.from_numpy(prng.spike_targets(350 + s, (B, 100, n))).to(DEV)
        loss = poisson_nll_mean(m(px), y)
        loss.backward()
        opt.step()
        sched.step()
        opt.zero_grad()
        losses.append(loss.item())
    ref = fx["curve_frozen" if frozen else "curve_train"]
    np.testing.assert_allclose(losses, ref, rtol=1e-3)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_mse_head_trains_like_torch_reference(dtype):
    """`training.loss: mse` through the Trainer loop (base.py:144-159 with MSELoss as criterion):
    3 steps of the small ViT (trainable encoder) against the CPU oracle's forward + MSE mean +
    torch AdamW / OneCycleLR on the same seeded batches and weights."""
    from vspike import FusedAdamW
    from vspike.trainer import Trainer
    cfg, B, n = cpu_ref.VIT_SMALL_FIXTURE, 2, 16
    m = _vit_model(cfg, 64, n, dtype=dtype)
    opt = FusedAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-5, weight_decay=0.01, eps=1e-8)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, total_steps=3, max_lr=1e-5, pct_start=0.15, div_factor=10)
    trainer = Trainer(m, opt, sched, config={"training": {"loss": "mse"}})
    batches = [(cpu_ref.make_pixels(cfg, B, seed=800 + s), prng.spike_targets(850 + s, (B, 100, n))) for s in range(3)]
    losses = [float(trainer.step(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV))) for x, y in batches]
    P = cpu_ref.to_torch(cpu_ref.make_vit_params(cfg, 64, n))
    fwd = lambda x, PP: cpu_ref.videomae_plugin_forward(x, PP, cfg, freeze_encoder=False)  # noqa: E731
    ref = cpu_ref.train_curve(fwd, P, [(torch.from_numpy(x), torch.from_numpy(y)) for x, y in batches], lr=1e-5,
                              criterion=cpu_ref.mse_mean)
    print(f"\n[{dtype}] mse curve {losses} ref {ref}")
    np.testing.assert_allclose(losses, ref, rtol=1e-3 if dtype == "fp32" else 1e-2)


def test_linear_plugin_matches_reference(golden):
    from vspike import Linear, poisson_nll_mean
    fx = golden("linear_f.npz")
    B, T, HW, n = 4, 8, 64, 16
    conf = {"model_class": "Linear",
            "encoder": {"input_dim": T * HW * HW, "hidden_dims": [256, 128], "output_dim": 64, "layer_num": 2},
            "decoder": {"input_dim": 64, "hidden_dims": [128, 256], "output_dim": 100 * n, "layer_num": 2}}
    m = Linear(conf)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    m.load_state_dict({k: torch.from_numpy(v) for k, v in cpu_ref.make_linear_params(shapes).items()})
    m = m.to(DEV)
    video = np.floor(prng.uniform(0, B * T * HW * HW, "video") * 256.0).astype(np.float32).reshape(B, T, 1, HW, HW)
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n))).to(DEV)
    out = m(torch.from_numpy(video).to(DEV))
    assert _maxrel(out.detach().cpu(), fx["log_rates"]) < 1e-4
    loss = poisson_nll_mean(out, y)
    assert abs(loss.item() - fx["loss"][0]) < 1e-5
    loss.backward()
    for k, p in m.named_parameters():
        ok, msg = cpu_ref.compare_summary(k, p.grad.cpu().numpy(), fx, rtol=1e-3, atol=1e-8)
        assert ok, msg


def test_linear_loss_curve_matches_reference(golden):
    from vspike import FusedAdamW, Linear, poisson_nll_mean
    fx = golden("linear_f.npz")
    B, T, HW, n = 4, 8, 64, 16
    conf = {"model_class": "Linear",
            "encoder": {"input_dim": T * HW * HW, "hidden_dims": [256, 128], "output_dim": 64, "layer_num": 2},
            "decoder": {"input_dim": 64, "hidden_dims": [128, 256], "output_dim": 100 * n, "layer_num": 2}}
    m = Linear(conf)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    m.load_state_dict({k: torch.from_numpy(v) for k, v in cpu_ref.make_linear_params(shapes).items()})
    m = m.to(DEV)
    opt = FusedAdamW(m.parameters(), lr=1e-6, weight_decay=0.01, eps=1e-8)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, total_steps=5, max_lr=1e-6, pct_start=0.15, div_factor=10)
    losses = []
    for s in range(5):
        v = np.floor(prng.uniform(100 + s, B * T * HW * HW, "video") * 256.0).astype(np.float32)
        y = torch.from_numpy(prng.spike_targets(200 + s, (B, 100, n))).to(DEV)
        loss = poisson_nll_mean(m(torch.from_numpy(v.reshape(B, T, 1, HW, HW)).to(DEV)), y)
        loss.backward()
        opt.step()
        sched.step()
        opt.zero_grad()
        losses.append(loss.item())
    np.testing.assert_allclose(losses, fx["curve"], rtol=1e-3)


def test_vit_bf16_trains_and_matches_fp32_gradients_direction():
    """bf16 mode at a larger size: gradients agree with the fp32 mode's (cosine > 0.99)."""
    from vspike import poisson_nll_mean
    cfg = cpu_ref.ViTCfg(hidden_size=192, num_attention_heads=3, intermediate_size=768, num_hidden_layers=2)
    B, n = 2, 8
    m32 = _vit_model(cfg, 64, n, dtype="fp32")
    m16 = _vit_model(cfg, 64, n, dtype="bf16")
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B)).to(DEV)
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n))).to(DEV)
    for m in (m32, m16):
        poisson_nll_mean(m(px), y).backward()
    for a, b in ((m32.enc_flat.grad, m16.enc_flat.grad), (m32.head_flat.grad, m16.head_flat.grad)):
        cos = torch.nn.functional.cosine_similarity(a.double(), b.double(), dim=0).item()
        assert cos > 0.99, cos


def test_state_dict_roundtrip_and_pickle(tmp_path):
    cfg = cpu_ref.VIT_SMALL_FIXTURE
    m = _vit_model(cfg, 64, 16)
    sd = m.reference_state_dict(modern_names=True)
    ref = cpu_ref.make_vit_params(cfg, 64, 16)
    for k, v in ref.items():
        assert np.array_equal(sd[k].cpu().numpy(), v), k
    torch.save({"model": m, "epoch": 0}, tmp_path / "m.pt")      # src/trainer/base.py:285-291
    m2 = torch.load(tmp_path / "m.pt", weights_only=False)["model"]    # our own file
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, 1)).to(DEV)
    with torch.no_grad():
        a, b = m(px), m2(px)
    # not bit-exact: the split-K head GEMM sums with f32 atomics in arrival order
    assert (a - b).abs().max().item() <= 1e-5 * a.abs().max().item()


def test_cached_buffers_two_forwards_before_backward():
    """The forward arena is cached per shape and reserved while its autograd state is alive: two
    forwards before one backward (and a no-grad forward in between) must give the gradients of
    separate passes."""
    from vspike import poisson_nll_mean
    cfg, B, n = cpu_ref.VIT_SMALL_FIXTURE, 2, 16
    m = _vit_model(cfg, 64, n)
    px1 = torch.from_numpy(cpu_ref.make_pixels(cfg, B)).to(DEV)
    px2 = px1.flip(0).contiguous() * 0.5
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n))).to(DEV)
    grads = []
    for x in (px1, px2):
        m.zero_grad(set_to_none=True)
        poisson_nll_mean(m(x), y).backward()
        grads.append((m.enc_flat.grad.clone(), m.head_flat.grad.clone()))
    m.zero_grad(set_to_none=True)
    o1 = m(px1)
    o2 = m(px2)
    with torch.no_grad():
        o3 = m(px1)
    assert torch.equal(o3, o1.detach())
    (poisson_nll_mean(o1, y) + poisson_nll_mean(o2, y)).backward()
    for k, g in enumerate((m.enc_flat.grad, m.head_flat.grad)):
        want = grads[0][k] + grads[1][k]
        assert float((g - want).norm() / want.norm()) < 1e-5
    # outputs handed to the caller are not overwritten by later steps
    o1c = o1.detach().clone()
    m(px2)
    assert torch.equal(o1.detach(), o1c)


def test_pixels_modified_before_backward_are_refused():
    """bf16 training gathers the pixels again in the patch-embedding weight gradient (no cols saved):
    an in-place write to the caller's input between forward and backward must raise (as autograd
    does for a modified saved tensor) instead of giving the next batch's gradient."""
    from vspike import poisson_nll_mean
    cfg, B, n = cpu_ref.VIT_SMALL_FIXTURE, 2, 16
    m = _vit_model(cfg, 64, n, dtype="bf16")
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B)).to(DEV)
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n))).to(DEV)
    poisson_nll_mean(m(px), y).backward()              # unchanged input: fine
    loss = poisson_nll_mean(m(px), y)
    px.mul_(0.5)                                       # a loader refilling its buffer in place
    with pytest.raises(RuntimeError, match="modified in place"):
        loss.backward()


def test_eval_epoch_matches_reference_eval_flow():
    """Trainer.eval_epoch (src/trainer/base.py:161-206) on two sessions: eval_loss and the
    per-session bps / rsquared means against the CPU restatement of the same flow."""
    from vspike.trainer import Trainer
    from oracle import metrics_ref
    cfg, B, n = cpu_ref.VIT_SMALL_FIXTURE, 2, 16
    m = _vit_model(cfg, 64, n)
    batches = []
    for eid in ("s0", "s1"):
        for k in range(3):                       # 6 trials per session <= 16 neurons
            px = torch.from_numpy(cpu_ref.make_pixels(cfg, B)).to(DEV) * (1 + 0.1 * k)
            y = torch.from_numpy(prng.spike_targets(40 + k + (10 if eid == "s1" else 0), (B, 100, n))).to(DEV)
            batches.append({"video": px, "ap": y, "eid": [eid] * B})
    res = Trainer(m, None).eval_epoch(batches)
    losses, sess = [], {}
    with torch.no_grad():
        for b in batches:
            out = m(b["video"])
            x, t = out.double(), b["ap"].double()
            losses.append(float((torch.exp(x) - t * x).mean()))
            s = sess.setdefault(b["eid"][0], ([], []))
            s[0].append(b["ap"].cpu().numpy())
            s[1].append(out.cpu().numpy())
    want = {"bps": [], "rsquared": []}
    for gts, outs in sess.values():
        r = metrics_ref.eval_session(np.concatenate(gts), np.concatenate(outs), dtype=np.float64)
        for k in want:
            want[k].append(r[k])
    assert abs(res["eval_loss"] - round(float(np.mean(losses)), 5)) <= 1e-5
    for k in want:
        assert abs(res[f"eval_{k}"] - round(float(np.mean(want[k])), 5)) <= 1e-5, (k, res, want)


@pytest.mark.parametrize("mode", [1, 2])
def test_deferred_side_stream_joins_give_identical_grads(mode):
    """VS_BWD_DEFER_JOIN / VS_BWD_DEFER_LAST only move where the caller's stream waits on the
    side-stream weight-gradient products; the products must equal those of a join at every block
    end over two steps (buffers reused across blocks).  The split-K dW sums are fixed-order, but the
    fused bias-gradient row sums add f32 atomics in arrival order, so the bar is 1e-5 of the norm
    (a read of a half-overwritten buffer would be off by O(1))."""
    import vspike.vit as V
    from vspike import poisson_nll_mean
    cfg, B, n = cpu_ref.VIT_SMALL_FIXTURE, 2, 16
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B)).to(DEV)
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n))).to(DEV)
    grads = {}
    old = V._DEFER
    try:
        for m_ in (0, mode):
            V._DEFER = m_
            m = _vit_model(cfg, 64, n, dtype="bf16")
            for _ in range(2):
                m.enc_flat.grad = None
                poisson_nll_mean(m(px), y).backward()
            torch.cuda.synchronize()
            grads[m_] = m.enc_flat.grad.detach().cpu().clone()
    finally:
        V._DEFER = old
    assert (grads[0] - grads[mode]).norm().item() <= 1e-5 * grads[0].norm().item()


def test_side_stream_off_gives_identical_grads():
    """VideoMAE.set_side_stream(False) (bench.py's instrumented pass: every weight-gradient product
    in order on the caller's stream) computes the same gradients as the default side stream, on the
    same model across the switch (the cached per-block structs are rebuilt)."""
    from vspike import poisson_nll_mean
    cfg, B, n = cpu_ref.VIT_SMALL_FIXTURE, 2, 16
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B)).to(DEV)
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n))).to(DEV)
    m = _vit_model(cfg, 64, n, dtype="bf16")
    grads = []
    for side in (True, False, True):
        m.set_side_stream(side)
        m.enc_flat.grad = None
        m.head_flat.grad = None
        poisson_nll_mean(m(px), y).backward()
        torch.cuda.synchronize()
        grads.append((m.enc_flat.grad.detach().clone(), m.head_flat.grad.detach().clone()))
    for g in grads[1:]:
        assert (g[0] - grads[0][0]).norm().item() <= 1e-6 * grads[0][0].norm().item()
        assert (g[1] - grads[0][1]).norm().item() <= 1e-6 * grads[0][1].norm().item()


def test_bf16_shadows_written_by_fused_adamw():
    """FusedAdamW rewrites the bf16 weight shadows in its update pass (vs_adamw param_lp): after
    each step they equal the rounded master weights, and an autograd-visible in-place write to a
    parameter makes the next forward re-cast."""
    from vspike import FusedAdamW, poisson_nll_mean
    cfg, B, n = cpu_ref.VIT_SMALL_FIXTURE, 2, 16
    m = _vit_model(cfg, 64, n, dtype="bf16")
    opt = FusedAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3, weight_decay=0.01)
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B)).to(DEV)
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n))).to(DEV)
    for _ in range(2):
        poisson_nll_mean(m(px), y).backward()
        opt.step()
        opt.zero_grad()
        sh = m._lp_shadows(torch.device(DEV))
        assert torch.equal(sh["enc"][0], m.enc_flat.detach().to(torch.bfloat16))
        assert torch.equal(sh["head"][0], m.head_flat.detach().to(torch.bfloat16))
    with torch.no_grad():
        m.head_flat.mul_(0.5)
    out = m(px)
    assert torch.equal(sh["head"][0], m.head_flat.detach().to(torch.bfloat16))
    m2 = _vit_model(cfg, 64, n, dtype="bf16")
    with torch.no_grad():
        m2.enc_flat.copy_(m.enc_flat)
        m2.head_flat.copy_(m.head_flat)
    assert torch.equal(out, m2(px))


def test_bf16_backward_bitwise_reproducible():
    """Every reduction of the bf16 train step sums in a fixed order (split-K dW partials and bias
    sums, the head dZ split-K, LayerNorm dgamma/dbeta partial rows, the loss): two backward passes
    from the same state give bit-identical gradients (hidden 192: the vectorised LayerNorm path)."""
    from vspike import poisson_nll_mean
    cfg = cpu_ref.ViTCfg(image_size=112, num_frames=8, hidden_size=192, num_hidden_layers=2,
                         num_attention_heads=3, intermediate_size=768)
    B, n = 2, 16
    m = _vit_model(cfg, 64, n, dtype="bf16")
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B)).to(DEV)
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n))).to(DEV)
    grads = []
    for _ in range(3):
        m.zero_grad(set_to_none=True)
        poisson_nll_mean(m(px), y).backward()
        grads.append((m.enc_flat.grad.clone(), m.head_flat.grad.clone()))
    for g in grads[1:]:
        assert torch.equal(g[0], grads[0][0]) and torch.equal(g[1], grads[0][1])


def test_linear_video_real_first_layer():
    """§8(f) row 4: the Linear plugin at the real `linear_video` geometry (config/model/
    linear_video.yaml: 120 frames x 128 x 128 -> K = 1,966,080, a 503 M-parameter first layer),
    B = 2 clips: forward (skinny split-K) and every gradient against an fp64 reference of the same
    math (src/model/linear.py:10-56) on the device.  Tolerances: the fp32 north star (1e-4 of
    max|ref| on log-rates, 1e-3 of the norm on gradients)."""
    from vspike import Linear, poisson_nll_mean
    n = 16
    conf = {"model_class": "Linear",
            "encoder": {"input_dim": 120 * 128 * 128, "hidden_dims": [256, 128], "output_dim": 64, "layer_num": 2},
            "decoder": {"input_dim": 64, "hidden_dims": [128, 256], "output_dim": 100 * n, "layer_num": 2}}
    torch.manual_seed(5)
    m = Linear(conf).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(6)
    video = torch.randint(0, 256, (2, 120, 1, 128, 128), device=DEV, generator=g).float()
    y = torch.poisson(torch.full((2, 100, n), 0.3, device=DEV), generator=g)
    out = m(video)
    loss = poisson_nll_mean(out, y)
    loss.backward()
    torch.cuda.synchronize()
    # fp64 reference of linear.py:10-15 (ReLU between hidden layers only)
    ps = {k: p.detach().double().requires_grad_() for k, p in m.named_parameters()}
    h = video.flatten(1).double()
    for stack in ("encoder", "decoder"):
        idx = sorted(int(k.split(".")[2]) for k in ps if k.startswith(stack) and k.endswith(".weight"))
        for j, i in enumerate(idx):
            h = h @ ps[f"{stack}.layers.{i}.weight"].t() + ps[f"{stack}.layers.{i}.bias"]
            if j < len(idx) - 1:
                h = torch.relu(h)
    ref = h.reshape(2, 100, n)
    rl = (torch.exp(ref) - y.double() * ref).mean()
    rl.backward()
    assert float((out.detach().double() - ref.detach()).abs().max() / ref.detach().abs().max()) < 1e-4
    assert abs(loss.item() - rl.item()) < 1e-5 * abs(rl.item())
    for k, p in m.named_parameters():
        err = float((p.grad.double() - ps[k].grad).norm() / ps[k].grad.norm())
        assert err < 1e-3, (k, err)


def test_kernel_timers_per_product():
    """bench.py's roofline reads the libvspike timers: with every timer on, one bf16 train step of
    an L-layer encoder charges exactly L launches to each ViT-block product timer (fwd / dX / dW of
    qkv, proj, fc1, fc2), L to each attention timer, none of the block's GEMMs to the generic GEMM
    classes beyond the patch-embed and head products, and positive algorithmic bytes to each."""
    from vspike import _lib as L, ops, poisson_nll_mean
    cfg = cpu_ref.ViTCfg(image_size=112, num_frames=8, hidden_size=192, num_hidden_layers=3,
                         num_attention_heads=3, intermediate_size=768)
    m = _vit_model(cfg, 64, 16, dtype="bf16")
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, 2)).to(DEV)
    y = torch.from_numpy(prng.spike_targets(1, (2, 100, 16))).to(DEV)
    poisson_nll_mean(m(px), y).backward()        # warm caches outside the timed pass
    torch.cuda.synchronize()
    ops.timing_enable((1 << len(L.TIMER_NAMES)) - 1)
    try:
        m.zero_grad(set_to_none=True)
        poisson_nll_mean(m(px), y).backward()
        torch.cuda.synchronize()
        got = {name: ops.timing_collect(t, with_bytes=True) for t, name in enumerate(L.TIMER_NAMES)}
    finally:
        ops.timing_enable(0)
    Lh = cfg.num_hidden_layers
    fused = m._mlp_fused(2)          # D = 192 bf16: the fused MLP kernels replace fc1 / fc2 fwd and dx_fc2
    unused = {"fwd_fc1", "fwd_fc2", "dx_fc2"} if fused else {"fwd_mlp", "dx_mlp"}
    unused |= {"fp8_quant"}          # compute_dtype fp8 only
    unused |= {"conv_fwd", "conv_dx", "conv_dw", "bn"}   # the R3D encoder's (tests/test_gpu_r3d.py)
    for name in L.TIMER_NAMES[8:] + ("attn_fwd", "attn_bwd", "ln_bwd"):
        n, ms, nbytes = got[name]
        want = 0 if name in unused else (2 * Lh if name.startswith("ln_") else Lh)
        assert n == want, (name, n)
        if want:
            assert ms > 0 and nbytes > 0, (name, ms, nbytes)
    # LayerNorm forwards: LN1 + LN2 per layer, fewer where the fused MLP epilogue runs the next
    # block's LN1 (vs_mlp_fwd_ln) or the proj product runs LN2 (vs_gemm_ln_fwd)
    assert 1 <= got["ln_fwd"][0] <= 2 * Lh, got["ln_fwd"]
    # outside the block: patch-embed fwd + head (fwd, dX) in "gemm", patch dW + head dW in "gemm_dw"
    assert 0 < got["gemm"][0] <= 6 and 0 < got["gemm_dw"][0] <= 4, (got["gemm"], got["gemm_dw"])


@pytest.mark.parametrize("side", [True, False])
def test_fused_ln_backward_and_serial_schedule_match_default(side):
    """The opt-in schedules of the block backward (VS_BWD_FUSE_LN: dX product + LayerNorm' in one
    launch; VSPIKE_SIDE=0: no side stream) compute the same gradients as the default.  Geometry with
    M = B x 1568 = 9,408 token rows, so the fused row-slab path (M >= 8192) runs.  Bars: the serial
    schedule 2e-5 of each flat gradient's norm (same products, dgamma/dbeta partial rows grouped
    the same way); the fused LN' keeps dh in f32 on the chip while the default writes the bf16
    dh1 / dh2 the bf16 block uses everywhere else, so 3e-3 (one bf16 rounding of a gradient;
    measured 8.6e-4)."""
    import vspike.vit as V
    from vspike import poisson_nll_mean
    cfg = cpu_ref.ViTCfg(image_size=224, num_frames=16, hidden_size=192, num_hidden_layers=2,
                         num_attention_heads=3, intermediate_size=768)
    B, n = 6, 16
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B)).to(DEV)
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n))).to(DEV)
    grads = {}
    old = (V._LN_FUSE, V._SIDE)
    runs = {"default": (False, True), "fused": (True, side)}
    if not side:
        runs["serial"] = (False, False)
    try:
        for key, (fuse, sd) in runs.items():
            V._LN_FUSE, V._SIDE = fuse, sd
            m = _vit_model(cfg, 64, n, dtype="bf16")
            poisson_nll_mean(m(px), y).backward()
            torch.cuda.synchronize()
            grads[key] = (m.enc_flat.grad.detach().double().cpu(), m.head_flat.grad.detach().double().cpu())
    finally:
        V._LN_FUSE, V._SIDE = old
    for a, b in zip(grads["default"], grads["fused"]):
        assert (a - b).norm().item() <= 3e-3 * a.norm().item()
    if not side:
        for a, b in zip(grads["default"], grads["serial"]):
            assert (a - b).norm().item() <= 2e-5 * a.norm().item()
