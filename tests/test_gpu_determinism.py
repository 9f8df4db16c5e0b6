"""Run-to-run determinism and blindness to memory the kernels must not read.

Every kernel of the bf16 train step sums in a fixed order, so reruns on the same inputs are
bit-identical.  A kernel that reads uninitialised memory (rows past the last token, workspace it
did not write, the slack after a tensor) or races on LDS shows up here as a rerun that differs,
which the parity tolerances (3e-2 on bf16 attention gradients) could hide.  Each case runs with the
bytes around and after the operands filled twice over — NaN, then large finite values — and the
workspaces pre-filled with NaN: the outputs must be finite and bit-identical across every rerun.
"""
import pytest
import torch

from oracle import cpu_ref, prng

pytestmark = pytest.mark.gpu
DEV = "cuda"
FILLS = (float("nan"), 3.0e4)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _padded(src, fill, extra_rows=64):
    """`src` copied to the device inside a buffer with `extra_rows` rows of `fill` after it."""
    buf = torch.full((src.shape[0] + extra_rows,) + tuple(src.shape[1:]), fill, dtype=src.dtype, device=DEV)
    buf[:src.shape[0]].copy_(src)
    return buf[:src.shape[0]]


@pytest.mark.parametrize("variant", [0, 0x90])
@pytest.mark.parametrize("shape", [(2, 196, 2), (4, 196, 2), (3, 33, 1), (1, 1568, 3), (2, 3136, 1)])
def test_attention_reruns_bitwise(knobs, variant, shape):
    """attn_fwd + attn_bwd (bf16) three times per fill: O, LSE and dQKV bit-identical and finite.
    (2, 196, 2) is test_gpu_dp.py's per-rank shape: 196 tokens = 1 full + 1 partial 128-row block."""
    from vspike import ops
    knobs("attn_variant", variant)
    B, N, H = shape
    D = H * 64
    g = torch.Generator().manual_seed(31)
    qkv = (torch.randn(B * N, 3 * D, generator=g) * 1.5).to(torch.bfloat16)
    do = torch.randn(B * N, D, generator=g).to(torch.bfloat16)
    outs = []
    for fill in FILLS:
        qd, dd = _padded(qkv, fill), _padded(do, fill)
        for _ in range(3):
            o = _padded(torch.zeros(B * N, D, dtype=torch.bfloat16), fill)
            lse = torch.full((B * H * N + 256,), fill, device=DEV)[:B * H * N].view(B, H, N)
            ops.attn_fwd(qd, o, lse, B, N, H)
            dqkv = _padded(torch.zeros(B * N, 3 * D, dtype=torch.bfloat16), fill)
            ws = torch.full((ops.attn_bwd_workspace_bytes(B, N, H) // 4 + 64,), float("nan"), device=DEV)
            ops.attn_bwd(qd, o, dd, lse, dqkv, ws, B, N, H)
            torch.cuda.synchronize()
            outs.append((o.clone(), lse.clone(), dqkv.clone()))
    for t in outs[0]:
        assert torch.isfinite(t.float()).all()
    for k, run in enumerate(outs[1:], 1):
        for name, a, b in zip(("o", "lse", "dqkv"), run, outs[0]):
            assert torch.equal(a, b), (name, k, float((a.float() - b.float()).abs().max()))


@pytest.mark.parametrize("M", [392, 1568 + 7])
def test_fused_mlp_reruns_bitwise(M):
    """vs_mlp_fwd and vs_mlp_bwd_da (ViT-Tiny widths) on a ragged token count, operands followed by
    NaN / large rows: outputs bit-identical and finite across reruns."""
    from vspike import ops
    D, F = 192, 768
    if not ops.mlp_fused_ok(M, D, F):
        pytest.skip("fused MLP not taken at this shape")
    g = torch.Generator().manual_seed(32)
    h2 = torch.randn(M, D, generator=g).to(torch.bfloat16)
    w1 = (torch.randn(F, D, generator=g) * 0.08).to(torch.bfloat16).to(DEV)
    b1 = (torch.randn(F, generator=g) * 0.3).to(DEV)
    w2 = (torch.randn(D, F, generator=g) * 0.04).to(torch.bfloat16).to(DEV)
    b2 = (torch.randn(D, generator=g) * 0.3).to(DEV)
    y = torch.randn(M, D, generator=g)
    dy = torch.randn(M, D, generator=g).to(torch.bfloat16)
    outs = []
    for fill in FILLS:
        hd, yd, dyd = _padded(h2, fill), _padded(y, fill), _padded(dy, fill)
        for _ in range(2):
            out = _padded(torch.zeros(M, D), fill)
            da = _padded(torch.zeros(M, F, dtype=torch.bfloat16), fill)
            a = _padded(torch.zeros(M, F, dtype=torch.bfloat16), fill)
            ops.mlp_fwd(hd, w1, b1, w2, b2, yd, out)
            ops.mlp_bwd_da(hd, w1, b1, w2, dyd, da, a)
            torch.cuda.synchronize()
            outs.append((out.clone(), da.clone(), a.clone()))
    for t in outs[0]:
        assert torch.isfinite(t.float()).all()
    for k, run in enumerate(outs[1:], 1):
        for name, a_, b_ in zip(("out", "da", "a"), run, outs[0]):
            assert torch.equal(a_, b_), (name, k)


def _dp_model(layers=4, hidden=128, heads=2, inter=512, n=16):
    from vspike import VideoMAE
    cfg = cpu_ref.ViTCfg(image_size=112, num_frames=8, hidden_size=hidden, num_hidden_layers=layers,
                         num_attention_heads=heads, intermediate_size=inter)
    conf = {"model_class": "VideoMAE", "freeze_encoder": False, "compute_dtype": "bf16",
            "backbone": {k: getattr(cfg, k) for k in ("image_size", "patch_size", "num_channels", "num_frames",
                                                       "tubelet_size", "hidden_size", "num_hidden_layers",
                                                       "num_attention_heads", "intermediate_size")},
            "encoder": {"output_dim": 64}, "decoder": {"output_dim": 100 * n}}
    m = VideoMAE(conf).to(DEV)
    m.load_reference_state_dict({k: torch.from_numpy(v) for k, v in cpu_ref.make_vit_params(cfg, 64, n).items()})
    return cfg, m


@pytest.mark.parametrize("B,hidden,heads,inter", [(2, 128, 2, 512), (4, 128, 2, 512), (2, 192, 3, 768)])
def test_model_backward_fresh_buffers_bitwise(B, hidden, heads, inter):
    """The bf16 step of test_gpu_dp.py's model (and ViT-Tiny's widths) built four times, each time
    after the allocator's free blocks were filled with NaN / large values, so every activation arena,
    workspace and gradient buffer starts from different garbage: the gradients are bit-identical.
    The fifth build runs every weight-gradient product in order on the main stream (no side stream,
    no deferred joins): the same bits, so no product races the side stream for a buffer."""
    from vspike import poisson_nll_mean
    n = 16
    grads = []
    for rep in range(5):
        junk = torch.full((64 << 20,), FILLS[rep % 2], device=DEV)   # 256 MB of garbage, then freed
        del junk
        cfg, m = _dp_model(hidden=hidden, heads=heads, inter=inter, n=n)
        m.set_side_stream(rep < 4)
        px = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=701)).to(DEV)
        y = torch.from_numpy(prng.spike_targets(751, (B, 100, n))).to(DEV)
        m.zero_grad(set_to_none=True)
        poisson_nll_mean(m(px), y).backward()
        torch.cuda.synchronize()
        grads.append((m.enc_flat.grad.clone(), m.head_flat.grad.clone()))
        lay = m.layout
        del m
    assert torch.isfinite(grads[0][0]).all() and torch.isfinite(grads[0][1]).all()
    for k, (ge, gh) in enumerate(grads[1:], 1):
        diff = [name for name, s in lay.enc.slots.items()
                if not torch.equal(ge[s.offset:s.offset + s.numel], grads[0][0][s.offset:s.offset + s.numel])]
        assert torch.equal(ge, grads[0][0]), ("encoder", k, float((ge - grads[0][0]).abs().max()), diff)
        assert torch.equal(gh, grads[0][1]), ("head", k)
