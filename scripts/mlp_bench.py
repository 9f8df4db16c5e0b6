"""Time the fused MLP kernels alone at the bench shape (128 clips: M = 200,704 tokens, D = 192,
F = 768): vs_mlp_fwd, vs_mlp_fwd_ln, vs_mlp_bwd_da, median of 20 launches after 5 warm-ups (torch
events on the current stream).  VSPIKE_LIB selects a diagnostic build for A/B runs."""
import ctypes
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-spike_amd")]
from vspike import ops, _lib as L  # noqa: E402

DEV = "cuda"


def timeit(fn, n=20, warm=5):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    M = int(os.environ.get("MLP_M", 200704))
    D, F = 192, 768
    g = torch.Generator(device=DEV).manual_seed(0)
    h2 = torch.randn(M, D, device=DEV, generator=g).to(torch.bfloat16)
    w1 = (torch.randn(F, D, device=DEV, generator=g) * 0.08).to(torch.bfloat16)
    b1 = torch.randn(F, device=DEV, generator=g) * 0.3
    w2 = (torch.randn(D, F, device=DEV, generator=g) * 0.04).to(torch.bfloat16)
    b2 = torch.randn(D, device=DEV, generator=g) * 0.3
    y = torch.randn(M, D, device=DEV, generator=g)
    out = torch.empty(M, D, device=DEV)
    dy = torch.randn(M, D, device=DEV, generator=g).to(torch.bfloat16)
    da = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
    a = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
    gam, bet = torch.ones(D, device=DEV), torch.zeros(D, device=DEV)
    hn = torch.empty(M, D, dtype=torch.bfloat16, device=DEV)
    mean, rstd = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    lib = L.lib()

    def fwd_ln():
        L.check(lib.vs_mlp_fwd_ln(M, D, F, h2.data_ptr(), D, w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                                  b2.data_ptr(), y.data_ptr(), D, out.data_ptr(), D, gam.data_ptr(), bet.data_ptr(),
                                  ctypes.c_float(1e-12), hn.data_ptr(), D, mean.data_ptr(), rstd.data_ptr(),
                                  L.stream()), "vs_mlp_fwd_ln")
    flop = 4.0 * M * D * F
    for name, fn, nbytes in [
            ("fwd", lambda: ops.mlp_fwd(h2, w1, b1, w2, b2, y, out), M * D * 10.0),
            ("fwd_ln", fwd_ln, M * D * 12.0 + M * 8.0),
            ("bwd_da", lambda: ops.mlp_bwd_da(h2, w1, b1, w2, dy, da, a), M * D * 4.0 + M * F * 4.0)]:
        med, best = timeit(fn)
        print(f"[mlp {name}] M={M}: median {med:.1f} us (best {best:.1f}); {flop / med / 1e6:.0f} TFLOP/s, "
              f"{nbytes / med / 1e3:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
