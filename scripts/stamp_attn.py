"""Wave timeline of the bf16 attention forward from a -DVS_STAMP diagnostic build.

usage: VSPIKE_LIB=.../libvspike_stamp.so python scripts/stamp_attn.py
Prints the kernel span, wave lifetime percentiles, the spread of wave start times, and how many
waves each SIMD held at once (from HW_ID: cu, simd, se, xcc).
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))
import torch  # noqa: E402

from vspike import _lib as L, ops  # noqa: E402


def main():
    B, N, H = int(os.environ.get("B", 16)), int(os.environ.get("N", 1568)), 3
    D = H * 64
    qkv = (torch.randn(B * N, 3 * D, device="cuda") * 1.5).to(torch.bfloat16)
    o = torch.empty(B * N, D, dtype=torch.bfloat16, device="cuda")
    lse = torch.empty(B, H, N, device="cuda")
    for _ in range(5):
        ops.attn_fwd(qkv, o, lse, B, N, H)
    torch.cuda.synchronize()
    nw = ((N + 127) // 128) * H * B * 4
    buf = (ctypes.c_ulonglong * (8 * 8192))()
    lib = L.lib()
    assert lib.vs_dbg_stamps(buf, 8 * 8192) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8)[:nw].astype(np.int64)
    t0 = a[:, 0].min()
    st, en = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0   # microseconds (100 MHz ticks)
    life = en - st
    hw = a[:, 2]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = a[:, 3] & 15
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    print(f"waves {nw}  span {en.max():.1f} us  distinct CUs {len(np.unique(key))}")
    print("lifetime us  p0 %.1f p10 %.1f p50 %.1f p90 %.1f p100 %.1f" % tuple(np.percentile(life, [0, 10, 50, 90, 100])))
    print("start us     p0 %.1f p10 %.1f p50 %.1f p90 %.1f p100 %.1f" % tuple(np.percentile(st, [0, 10, 50, 90, 100])))
    # max concurrent waves per SIMD
    sk = key * 4 + simd
    mx = []
    for k in np.unique(sk):
        idx = np.where(sk == k)[0]
        ev = sorted([(st[i], 1) for i in idx] + [(en[i], -1) for i in idx], key=lambda x: (x[0], x[1]))
        c = m = 0
        for _, d in ev:
            c += d
            m = max(m, c)
        mx.append(m)
    mx = np.array(mx)
    print("waves per SIMD (total)   ", np.bincount(np.bincount(sk)))
    print("max concurrent per SIMD  ", np.bincount(mx))
    # timeline histogram: active waves in 10 bins
    bins = np.linspace(0, en.max(), 11)
    act = [int(((st <= t) & (en > t)).sum()) for t in (bins[:-1] + bins[1:]) / 2]
    print("active waves over time   ", act)
    tot = a[:, 6].astype(np.float64)
    print("shader cycles per wave p50 %.0f  (%.2f GHz)" % (np.median(tot), np.median(tot) / np.median(life) / 1e3))
    print("share in vmcnt wait p50 %.3f  barrier wait p50 %.3f" % (np.median(a[:, 4] / tot), np.median(a[:, 5] / tot)))


if __name__ == "__main__":
    main()
