"""MX-FP8 activation quantisation at C5's 128-clip geometry (M = 128 x 3,136 tokens, K = 768 / 3,072,
bf16 in): time per launch and HBM rate (2 B read + 1 B written per element + one scale byte per 32).
usage: python scripts/quant_bench.py [--reps 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))

import torch  # noqa: E402

from vspike import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rows", type=int, default=128 * 3136)
    a = ap.parse_args()
    for K in (768, 3072):
        M = a.rows
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        q = torch.empty(M, K, dtype=torch.uint8, device="cuda")
        s = torch.empty(M, K // 32, dtype=torch.uint8, device="cuda")
        for _ in range(3):
            ops.quant_mxfp8(x, q, s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.reps):
            ops.quant_mxfp8(x, q, s)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.reps * 1e3
        nbytes = M * K * 3 + M * K // 32
        print(f"quant M={M} K={K}: {us:.1f} us/launch, {nbytes / us / 1e6:.2f} TB/s", flush=True)
        del x, q, s


if __name__ == "__main__":
    main()
