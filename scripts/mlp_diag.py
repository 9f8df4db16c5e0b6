"""Diagnostic for the fused MLP backward (vs_mlp_bwd_da): where its da differs from the fp64
reference (non-finite or off) by token-in-block, feature-in-chunk and chunk."""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-spike_amd")]
from vspike import ops  # noqa: E402

DEV = "cuda"


def gelu(x):
    return 0.5 * x * (1.0 + torch.erf(x / 2 ** 0.5))


def gelu_grad(x):
    return 0.5 * (1.0 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5


for M, F in [(100, 768), (4096, 64), (25088, 768)]:
    D = 192
    g = torch.Generator(device=DEV).manual_seed(M + F + 1)
    h2 = torch.randn(M, D, device=DEV, generator=g).to(torch.bfloat16)
    w1 = (torch.randn(F, D, device=DEV, generator=g) * 0.08).to(torch.bfloat16)
    b1 = torch.randn(F, device=DEV, generator=g) * 0.3
    w2 = (torch.randn(D, F, device=DEV, generator=g) * 0.04).to(torch.bfloat16)
    dy = torch.randn(M, D, device=DEV, generator=g).to(torch.bfloat16)
    for variant in ("dy", "zero_dy", "ones_dy"):
        dyv = {"dy": dy, "zero_dy": torch.zeros_like(dy), "ones_dy": torch.ones_like(dy)}[variant]
        da = torch.full((M, F), 3.0, dtype=torch.bfloat16, device=DEV)
        a = torch.full((M, F), 3.0, dtype=torch.bfloat16, device=DEV)
        ops.mlp_bwd_da(h2, w1, b1, w2, dyv, da, a)
        torch.cuda.synchronize()
        pre = h2.double() @ w1.double().t() + b1.double()
        dref = dyv.double() @ w2.double()
        ref = dref * gelu_grad(pre)
        dd = da.double()
        bad_nf = ~torch.isfinite(dd)
        err = (dd - ref).abs()
        tol = 8e-3 * ref.abs().max().clamp_min(1e-30)
        bad = bad_nf | (err > tol)
        print(f"M={M} F={F} {variant}: a err {float((a.double() - gelu(pre)).abs().max()):.2e} "
              f"non-finite {int(bad_nf.sum())} off {int(bad.sum())} of {M * F}; "
              f"max|ref| {float(ref.abs().max()):.3e}", flush=True)
        if bad.any():
            idx = bad.nonzero()
            r, c = idx[:, 0], idx[:, 1]
            print("  token%32 hist:", torch.bincount(r % 32, minlength=32).tolist())
            print("  feat%64 hist:", torch.bincount(c % 64, minlength=64).tolist())
            print("  chunk hist:", torch.bincount(c // 64).tolist()[:16])
            print("  block hist (first 16):", torch.bincount(r // 32).tolist()[:16])
            for rr_, cc_ in idx[:6].tolist():
                # da / gelu'(pre) recovers the kernel's W2 product where gelu' is not small
                gg = float(gelu_grad(pre)[rr_, cc_])
                print(f"   ({rr_},{cc_}) da {float(dd[rr_, cc_])!r} ref {float(ref[rr_, cc_]):.4e} "
                      f"dref {float(dref[rr_, cc_]):.4e} gelu' {gg:.4e} pre {float(pre[rr_, cc_]):.4e}")
