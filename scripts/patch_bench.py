"""Time the patch embedding kernels at the bench batch: vs_patch_embed_fwd (fused gather GEMM) and
vs_patch_embed_dw (gather weight gradient), hipEvents on the launch stream, plus their algorithmic
bytes rates.  usage: python scripts/patch_bench.py [--batch 128] [--reps 20]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))
from vspike import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    B, F, C, H, W, D = a.batch, 16, 3, 224, 224, 192
    n_tok = (F // 2) * (H // 16) * (W // 16)
    M, K = B * n_tok, C * 512
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    px = torch.randn(B, F, C, H, W, device=dev, generator=g)
    w = (torch.randn(D, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
    bias = torch.randn(D, device=dev, generator=g)
    pos = torch.randn(n_tok, D, device=dev, generator=g)
    out = torch.empty(M, D, device=dev)
    dx = torch.randn(M, D, device=dev, generator=g).to(torch.bfloat16)
    dw = torch.zeros(D, K, device=dev)
    db = torch.zeros(D, device=dev)
    ws = torch.empty(ops.patch_embed_dw_workspace_bytes(M, D, K) // 4 + 4, device=dev)
    cases = {
        "patch_embed_fwd": (lambda: ops.patch_embed_fwd(px, w, bias, pos, out, 2, 16),
                            M * K * 4 + D * K * 2 + M * D * 4 + n_tok * D * 4),
        "patch_embed_dw": (lambda: ops.patch_embed_dw(px, dx, dw, db, 2, 16, workspace=ws),
                           M * K * 4 + M * D * 2 + D * K * 8),
    }
    for name, (fn, nbytes) in cases.items():
        for _ in range(3):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(a.reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / a.reps
        print(f"{name:18s} {us:8.1f} us  {nbytes / us / 1e3:7.1f} GB/s  (B = {B}, {nbytes / 1e6:.0f} MB)", flush=True)


if __name__ == "__main__":
    main()
