"""Phase timeline of the whole-K GEMM (qkv shape; N=768 EPI=gelu: fc1) from a -DVS_STAMP build.
usage: VSPIKE_LIB=.../libvspike_stamp.so [N=768 EPI=gelu] python scripts/stamp_gemm.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))
import torch  # noqa: E402

from vspike import _lib as L, ops  # noqa: E402


def main():
    M, K = 25088, 192
    N = int(os.environ.get("N", 576))
    x = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    pre = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    gelu = os.environ.get("EPI") == "gelu"   # fc1 + GELU (pre-activation written too)
    for _ in range(5):
        if gelu:
            ops.linear(x, w, y, bias=b, epilogue=L.EPI_GELU, aux_out=pre, ld_aux_out=N)
        else:
            ops.linear(x, w, y, bias=b)
    torch.cuda.synchronize()
    nblk = (M // 128) * ((N + 63) // 64)
    nw = nblk * 4
    buf = (ctypes.c_ulonglong * (8 * 8192))()
    assert L.lib().vs_dbg_gstamps(buf, 8 * 8192) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8)[:min(nw, 8192)].astype(np.int64)
    d = lambda i, j: a[:, j] - a[:, i]  # noqa: E731
    for name, i, j in (("issue DMA", 0, 1), ("wait DMA + barrier", 1, 2), ("MFMA", 2, 3), ("epilogue", 3, 4),
                       ("total", 0, 4)):
        v = d(i, j)
        print(f"{name:22s} cycles p10 {np.percentile(v, 10):8.0f} p50 {np.percentile(v, 50):8.0f} p90 {np.percentile(v, 90):8.0f}")
    rt = (a[:, 6] - a[:, 6].min()) / 100.0
    print("block end times (us) p10/p50/p90/max", np.percentile(rt, [10, 50, 90, 100]))


if __name__ == "__main__":
    main()
