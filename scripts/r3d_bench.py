"""The C4 sub-record of bench.py alone (R3D-18, 32x112x112, n = 256, fp32): one JSON line.
Usage: python scripts/r3d_bench.py [--batch 16] [--steps 10] [--no-check]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--profile-steps", type=int, default=2)
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()
    args = argparse.Namespace(c4_batch=a.batch, c4_steps=a.steps, c4_warmup=a.warmup,
                              c4_profile_steps=a.profile_steps, no_cpu_baseline=a.no_check)
    torch.cuda.set_device(0)
    print(json.dumps(bench.c4_subrecord(args, 1, 0, torch.device("cuda", 0))), flush=True)


if __name__ == "__main__":
    main()
