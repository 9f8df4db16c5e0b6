"""Phase timeline of the row-panel GEMM from a -DVS_STAMP build (shape via env M N K, BKC=0/1).
usage: VSPIKE_LIB=.../libvspike_stamp.so python scripts/stamp_panel.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))
import torch  # noqa: E402

from vspike import _lib as L, ops  # noqa: E402


def main():
    M, N, K = (int(os.environ.get(k, v)) for k, v in (("M", 25088), ("N", 192), ("K", 192)))
    x = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.5).to(torch.bfloat16)
    y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    for _ in range(5):
        ops.linear(x, w, y)
    torch.cuda.synchronize()
    items = (M + 127) // 128 * (N // 64)
    G = min(items, 512)
    nw = G * 4
    buf = (ctypes.c_ulonglong * (8 * 8192))()
    assert L.lib().vs_dbg_gstamps(buf, 8 * 8192) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8)[:min(nw, 8192)].astype(np.int64)
    d = lambda i, j: a[:, j] - a[:, i]  # noqa: E731
    for name, i, j in (("first W image", 0, 1), ("first MFMA+stage", 1, 2), ("rest items", 2, 3),
                       ("last epilogue", 3, 4), ("total", 0, 4)):
        v = d(i, j)
        print(f"{name:20s} cycles p10 {np.percentile(v, 10):8.0f} p50 {np.percentile(v, 50):8.0f} p90 {np.percentile(v, 90):8.0f}")
    st = (a[:, 7] - a[:, 7].min()) / 100.0
    en = (a[:, 6] - a[:, 7].min()) / 100.0
    print("wave start us p0/p50/p90/max", np.percentile(st, [0, 50, 90, 100]))
    print("wave end   us p0/p50/p90/max", np.percentile(en, [0, 50, 90, 100]))
    print("lifetime   us p10/p50/p90", np.percentile(en - st, [10, 50, 90]))


if __name__ == "__main__":
    main()
