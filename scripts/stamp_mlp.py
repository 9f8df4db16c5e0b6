"""Where the fused MLP forward's time goes, per wave (diagnostic build with -DVS_MLP_STAMP):
total cycles, cycles at the chunk-start wait (weight DMA landed + barrier), epilogue cycles, chunks.

usage: python scripts/variant_build.py stamp VS_MLP_STAMP mlp.hip
       VSPIKE_LIB=video-spike_amd/vspike/_build/libvspike_stamp.so python scripts/stamp_mlp.py
"""
import ctypes
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-spike_amd")]
from vspike import ops, _lib as L  # noqa: E402


def main():
    M, D, F = int(os.environ.get("MLP_M", 200704)), 192, 768
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    h2 = torch.randn(M, D, device=dev, generator=g).to(torch.bfloat16)
    w1 = (torch.randn(F, D, device=dev, generator=g) * 0.08).to(torch.bfloat16)
    b1 = torch.randn(F, device=dev, generator=g) * 0.3
    w2 = (torch.randn(D, F, device=dev, generator=g) * 0.04).to(torch.bfloat16)
    b2 = torch.randn(D, device=dev, generator=g) * 0.3
    y = torch.randn(M, D, device=dev, generator=g)
    out = torch.empty(M, D, device=dev)
    for _ in range(5):
        ops.mlp_fwd(h2, w1, b1, w2, b2, y, out)
    torch.cuda.synchronize()
    lib = L.lib()
    lib.vs_dbg_mlp_stamps.restype = ctypes.c_int
    n = 4 * 4096
    buf = (ctypes.c_ulonglong * n)()
    assert lib.vs_dbg_mlp_stamps(buf, n) == 0
    rows = [tuple(buf[4 * w:4 * w + 4]) for w in range(4096) if buf[4 * w + 3] > 0]
    tot = sum(r[0] for r in rows) / len(rows)
    wait = sum(r[1] for r in rows) / len(rows)
    epi = sum(r[2] for r in rows) / len(rows)
    ch = sum(r[3] for r in rows) / len(rows)
    print(f"[mlp stamp] waves {len(rows)}: total {tot:.0f} cyc, chunk-start wait {wait:.0f} ({wait / tot:.1%}), "
          f"epilogue {epi:.0f} ({epi / tot:.1%}), rest {tot - wait - epi:.0f}; chunks {ch:.1f} -> "
          f"{(tot - wait - epi) / ch:.0f} cyc of compute per chunk, {wait / ch:.0f} waiting", flush=True)
    mx = max(r[0] for r in rows)
    print(f"[mlp stamp] slowest wave {mx} cyc; max wait {max(r[1] for r in rows)}", flush=True)


if __name__ == "__main__":
    main()
