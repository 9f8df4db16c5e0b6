"""BASELINE C5 at its stated precision: ViT-Base width at 32 frames (3,136 tokens), n = 1,024, with the
block's four Linear forwards on MX-FP8 (compute_dtype "fp8": vs_gemm_mxfp8 via the block executor;
everything else bf16, the backward bf16), against the reference's own encoder + head (fixture
vit_base32f from the HF VideoMAEModel the reference plugin executes: oracle/gen_fixtures.py).

The bars are the fp8 format's, documented here: e4m3 keeps 3 mantissa bits (2^-4 relative per
element, 16x bf16's), so the block outputs carry ~1-2 % relative noise; log-rates FP8_OUT of
max |ref|, loss FP8_LOSS relative, gradients FP8_GRAD norm-relative (the bf16 backward runs on the
fp8 forward's activations).  Measured values are printed with -s.

The tight check is test_c5_fp8_matches_the_mx_reference: the same encoder with the MX-FP8 round trip
applied to the four products' operands in the reference too (oracle/cpu_ref.py mx_matmul, the recipe
test_gpu_fp8.py pins byte for byte against vs_quant_mxfp8), so what is left is the bf16 path's own
noise — bars of the bf16 path's size, not the format's.

C5's temporal transformer has no reference code: nothing to pin it against,
so it is not built.
"""
import os
import numpy as np
import pytest
import torch

from oracle import cpu_ref, prng

pytestmark = pytest.mark.gpu
DEV = "cuda"

# ~2x the values measured on MI355X (oracle/tolerances.py, shared with bench.py's fp8 parity leg)
from oracle.tolerances import FP8_GRAD, FP8_LOSS, FP8_OUT  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _model(cfg, n, dtype):
    from vspike import VideoMAE
    conf = {"model_class": "VideoMAE", "freeze_encoder": False, "compute_dtype": dtype,
            "backbone": {k: getattr(cfg, k) for k in ("image_size", "patch_size", "num_channels", "num_frames",
                                                       "tubelet_size", "hidden_size", "num_hidden_layers",
                                                       "num_attention_heads", "intermediate_size",
                                                       "layer_norm_eps")},
            "encoder": {"output_dim": 64}, "decoder": {"output_dim": 100 * n}}
    m = VideoMAE(conf).to(DEV)
    m.load_reference_state_dict({k: torch.from_numpy(v) for k, v in cpu_ref.make_vit_params(cfg, 64, n).items()})
    return m


def test_c5_fp8_encoder_geometry_forward_backward(golden):
    from vspike import poisson_nll_mean, _lib as L
    from vspike.layout import modern_name
    fx = golden("vit_base32f.npz")
    cfg, B, n = cpu_ref.ViTCfg(num_frames=32, num_hidden_layers=1), 1, 1024
    m = _model(cfg, n, "fp8")
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=32)).to(DEV)
    y = torch.from_numpy(prng.spike_targets(32, (B, 100, n))).to(DEV)
    L.dispatch_reset()
    out = m(px)
    loss = poisson_nll_mean(out, y)
    loss.backward()
    torch.cuda.synchronize()
    counts = L.dispatch_counts()
    assert counts["gemm_fp8"] == 4 * cfg.num_hidden_layers, counts      # qkv, proj, fc1, fc2 on MX-FP8
    out_err = float(np.abs(out.detach().cpu().numpy() - fx["log_rates"]).max() / np.abs(fx["log_rates"]).max())
    loss_err = abs(loss.item() - fx["loss"][0]) / abs(fx["loss"][0])
    shapes = cpu_ref.vit_param_shapes(cfg, 64, n)
    errs = {}
    for name, which, slot, rows in m.layout.hf_items():
        flat = m.enc_flat.grad if which == "enc" else m.head_flat.grad
        t = (m.layout.enc if which == "enc" else m.layout.head).view(flat, slot)
        k = modern_name(name)
        g = (t if rows is None else t[rows]).detach().cpu().numpy().reshape(shapes[k])
        errs[k] = cpu_ref.summary_rel_error(k, g, fx)
    worst = max(errs, key=errs.get)
    print(f"\n[C5 fp8] log-rate err {out_err:.3e}  loss err {loss_err:.3e}  worst grad {worst} {errs[worst]:.3e}")
    assert out_err < FP8_OUT and loss_err < FP8_LOSS
    bad = {k: v for k, v in errs.items() if v > FP8_GRAD}
    assert not bad, bad


def test_c5_fp8_is_closer_to_the_reference_than_a_wrong_model(golden):
    """Guard against a bar that passes anything: the fp8 model's log-rates (quantisation noise in all
    four block products) must be closer to the reference than those of the bf16 model with ONE
    product systematically wrong by 10 % (fc1's weight scaled by 1.1) — the size of error a
    mis-applied block scale or a dropped term would cause."""
    fx = golden("vit_base32f.npz")
    cfg, B, n = cpu_ref.ViTCfg(num_frames=32, num_hidden_layers=1), 1, 1024
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=32)).to(DEV)
    ref = fx["log_rates"]
    with torch.no_grad():
        good = _model(cfg, n, "fp8")(px).cpu().numpy()
        mb = _model(cfg, n, "bf16")
        plain = mb(px).cpu().numpy()
        w = mb.layout.enc.view(mb.enc_flat, "0.w_fc1")
        w.mul_(1.1)
        mb.invalidate_lp()
        bad = mb(px).cpu().numpy()
    e_good = np.abs(good - ref).max() / np.abs(ref).max()
    e_bf16 = np.abs(plain - ref).max() / np.abs(ref).max()
    e_bad = np.abs(bad - ref).max() / np.abs(ref).max()
    print(f"\n[C5 fp8] err {e_good:.3e}; bf16 {e_bf16:.3e}; bf16 with fc1 x 1.1 {e_bad:.3e}")
    assert e_bf16 < e_good < e_bad


# vs the MX-aware reference: ~2x the values measured on MI355X (printed with -s)
from oracle.tolerances import FP8_MX_GRAD as MX_GRAD, FP8_MX_LOSS as MX_LOSS, FP8_MX_OUT as MX_OUT  # noqa: E402


def test_c5_fp8_matches_the_mx_reference():
    """The fp8 model against a reference that applies the SAME quantisation (the four block products on
    MX-FP8 round trips of bf16 operands, straight-through backward) in f32 on the CPU: log-rates,
    loss and every gradient (norm-relative).  The errors must also be well under the plain
    reference's (test above), i.e. the fp8 path's distance from fp32 is the format's and nothing else."""
    from vspike import poisson_nll_mean
    from vspike.layout import modern_name
    cfg, B, n = cpu_ref.ViTCfg(num_frames=32, num_hidden_layers=1), 1, 1024
    params = cpu_ref.make_vit_params(cfg, 64, n)
    px = cpu_ref.make_pixels(cfg, B, seed=32)
    y = prng.spike_targets(32, (B, 100, n))
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    P = cpu_ref.to_torch(params)
    ref = cpu_ref.videomae_plugin_forward(torch.from_numpy(px), P, cfg, freeze_encoder=False, mm=cpu_ref.mx_matmul)
    lref = cpu_ref.poisson_nll_mean(ref, torch.from_numpy(y))
    lref.backward()
    plain = cpu_ref.videomae_plugin_forward(torch.from_numpy(px), cpu_ref.to_torch(params, requires_grad=False),
                                            cfg, freeze_encoder=False).detach()

    m = _model(cfg, n, "fp8")
    out = m(torch.from_numpy(px).to(DEV))
    loss = poisson_nll_mean(out, torch.from_numpy(y).to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    o = out.detach().cpu()
    r = ref.detach()
    out_err = float((o - r).abs().max() / r.abs().max())
    plain_err = float((o - plain).abs().max() / plain.abs().max())
    loss_err = abs(loss.item() - lref.item()) / abs(lref.item())
    errs = {}
    for name, which, slot, rows in m.layout.hf_items():
        flat = m.enc_flat.grad if which == "enc" else m.head_flat.grad
        t = (m.layout.enc if which == "enc" else m.layout.head).view(flat, slot)
        k = modern_name(name)
        g = (t if rows is None else t[rows]).detach().cpu().double().reshape(P[k].shape)
        gr = P[k].grad.double()
        errs[k] = float((g - gr).norm() / gr.norm().clamp_min(1e-30))
    worst = max(errs, key=errs.get)
    print(f"\n[C5 fp8 vs MX reference] log-rate err {out_err:.3e} (vs plain f32 reference {plain_err:.3e})  "
          f"loss err {loss_err:.3e}  worst grad {worst} {errs[worst]:.3e}")
    assert out_err < MX_OUT and loss_err < MX_LOSS, (out_err, loss_err)
    assert out_err < 0.5 * plain_err, (out_err, plain_err)
    bad = {k: v for k, v in errs.items() if v > MX_GRAD}
    assert not bad, bad
