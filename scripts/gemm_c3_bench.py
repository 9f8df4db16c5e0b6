"""C3 block products at the bench's 128 clips (M = 200,704 token rows, D = 768, F = 3072): vs_gemm
(the dispatch the step takes) against torch.matmul (hipBLASLt, the library yardstick: guide §5.4 rule
10 — a ceiling needs a known-good reference on the same hardware), random bf16 operands, hipEvents.
Usage: python scripts/gemm_c3_bench.py [--reps 10] [--only fwd|dx|dw] [--rows 200704]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from vspike import _lib as L, ops  # noqa: E402

PEAK = 2.5e15


def timeit(fn, reps):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--rows", type=int, default=200704)
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--dw-nobias", action="store_true", help="dW products without the fused bias gradient")
    a = ap.parse_args()
    M, D, F = a.rows, 768, 3072
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16

    def rnd(*s, scale=1.0):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(bf)
    # name: (N, K, epilogue, out dtype, b_kcontig)
    fwd = {"fwd_qkv": (3 * D, D, L.EPI_BIAS, bf, True), "fwd_proj": (D, D, L.EPI_BIAS | L.EPI_RESIDUAL, torch.float32, True),
           "fwd_fc1": (F, D, L.EPI_BIAS | L.EPI_GELU | L.EPI_GELU_GRAD, bf, True),
           "fwd_fc2": (D, F, L.EPI_BIAS | L.EPI_RESIDUAL, torch.float32, True),
           "dx_fc2": (F, D, L.EPI_MUL_AUX, bf, False), "dx_fc1": (D, F, 0, torch.float32, False),
           "dx_proj": (D, D, 0, bf, False), "dx_qkv": (D, 3 * D, 0, torch.float32, False)}
    print(f"M = {M}; TF/s and fraction of the 2.5 PF bf16 roof; torch = torch.matmul (hipBLASLt) plain product")
    for name, (N, K, epi, odt, bkc) in fwd.items():
        if a.only and not name.startswith(a.only):
            continue
        x = rnd(M, K)
        w = rnd(N, K, scale=K ** -0.5)
        wb = w if bkc else w.t().contiguous()
        out = torch.empty(M, N, dtype=odt, device=dev)
        bias = torch.randn(N, device=dev, generator=g)
        res = torch.randn(M, N, device=dev, generator=g) if epi & L.EPI_RESIDUAL else None
        aux_out = torch.empty(M, N, dtype=bf, device=dev) if epi & L.EPI_GELU else None
        aux_in = rnd(M, N) if epi & L.EPI_MUL_AUX else None
        kw = dict(M=M, N=N, K=K, a_kcontig=True, b_kcontig=bkc, lda=K, ldb=K if bkc else N, ldc=N, epilogue=epi,
                  bias=bias if epi & L.EPI_BIAS else None, residual=res, ld_residual=N if res is not None else 0,
                  aux_out=aux_out, ld_aux_out=N if aux_out is not None else 0, aux_in=aux_in,
                  ld_aux_in=N if aux_in is not None else 0)
        L.dispatch_reset()
        t_ours = timeit(lambda: ops.gemm(x, wb, out, **kw), a.reps)
        path = [k for k, v in L.dispatch_counts().items() if v]
        fl = 2.0 * M * N * K
        line = f"{name:10s} {M}x{N}x{K} ours {t_ours:8.1f} us {fl / t_ours / 1e6:7.1f} TF/s ({fl / t_ours / 1e6 / 2500:.3f}) {path}"
        if not a.no_torch:
            wt = w.t() if bkc else wb        # [K, N] view for torch
            t_t = timeit(lambda: torch.matmul(x, wt), a.reps)
            line += f" | torch {t_t:8.1f} us {fl / t_t / 1e6:7.1f} TF/s ({fl / t_t / 1e6 / 2500:.3f})"
        print(line, flush=True)
        del x, w, wb, out, res, aux_out, aux_in
    dw = {"dw_qkv": (3 * D, D), "dw_proj": (D, D), "dw_fc1": (F, D), "dw_fc2": (D, F)}
    for name, (Mo, No) in dw.items():
        if a.only and not name.startswith(a.only):
            continue
        dy = rnd(M, Mo)
        xx = rnd(M, No)
        c = torch.zeros(Mo, No, device=dev)
        db = torch.zeros(Mo, device=dev)
        ws = torch.empty(ops.splitk_workspace_bytes(bf, Mo, No, M) // 4 + 64, device=dev)
        L.dispatch_reset()
        dbb = None if a.dw_nobias else db
        t_ours = timeit(lambda: ops.linear_dw(dy, xx, c, db=dbb, workspace=ws), a.reps)
        path = [k for k, v in L.dispatch_counts().items() if v]
        fl = 2.0 * M * Mo * No
        line = f"{name:10s} {Mo}x{No}x{M} ours {t_ours:8.1f} us {fl / t_ours / 1e6:7.1f} TF/s ({fl / t_ours / 1e6 / 2500:.3f}) {path}"
        if not a.no_torch:
            t_t = timeit(lambda: torch.matmul(dy.t(), xx), a.reps)
            line += f" | torch {t_t:8.1f} us {fl / t_t / 1e6:7.1f} TF/s ({fl / t_t / 1e6 / 2500:.3f})"
        print(line, flush=True)
        del dy, xx, c, ws


if __name__ == "__main__":
    main()
