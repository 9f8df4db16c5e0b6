"""Attention forward time and safe-softmax re-run rate vs the logit scale at the bench grid (C2:
128 clips, H = 3, N = 1568), VERDICT r4 item 8.  Usage: python scripts/attn_logit_scale.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

from vspike import _lib as L, ops  # noqa: E402
from test_gpu_attn_logits import make_qkv  # noqa: E402


def main():
    B, N, H = 128, 1568, 3
    flop = 4.0 * B * H * N * N * 64
    nwg = B * H * ((N + 127) // 128)
    print(f"B={B} N={N} H={H}: {nwg} workgroups per launch")
    for smax, spiky in ((1.0, False), (10.0, False), (20.0, False), (30.0, False), (40.0, False), (38.0, True),
                        (50.0, False), (60.0, True), (60.0, False), (70.0, False), (90.0, False)):
        qkv = make_qkv(B, N, H, smax, spiky)
        o = torch.empty(B * N, H * 64, dtype=torch.bfloat16, device="cuda")
        lse = torch.empty(B, H, N, device="cuda")
        for _ in range(2):
            ops.attn_fwd(qkv, o, lse, B, N, H)
        torch.cuda.synchronize()
        L.attn_redo_count(reset=True)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        s.record()
        for _ in range(reps):
            ops.attn_fwd(qkv, o, lse, B, N, H)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / reps * 1e3
        redo = L.attn_redo_count(reset=True) / reps
        print(f"smax {smax:5.1f} {'spiky' if spiky else 'gauss'}: {us:8.1f} us  {flop / us / 1e6:7.1f} TF/s  "
              f"re-run {redo:7.1f} of {nwg} workgroups ({100 * redo / nwg:5.1f} %)", flush=True)


if __name__ == "__main__":
    main()
