"""Interleaved A/B of the R3D-18 (C4) train step over knob settings in ONE process
(cdna_hip_programming.md rule 24): rounds x variants, each timing `--steps` full train steps
(fwd + bwd + AdamW) after its own re-warm step, plus the per-class kernel times of one instrumented
step per variant (conv fwd / dX / dW, BN).

usage: python scripts/r3d_ab.py --knob conv_mfma --values 1,2 [--batch 16 --rounds 5 --steps 5]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", default="conv_mfma")
    ap.add_argument("--values", default="1,2")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    from vspike import _lib as L, ops
    from vspike.trainer import build_optimizer, Trainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    spec = {"model": "r3d18", "neurons": 256, "dtype": "fp32", "frames": None, "freeze": False, "lr": None,
            "loss": "poisson", "batch": a.batch}
    config, criterion, model, B, pixels, target = bench._setup(spec, dev, 0)
    opt, sched = build_optimizer(model, config, total_steps=10000, world=1)
    trainer = Trainer(model, opt, sched, criterion=criterion)
    values = [int(v, 0) for v in a.values.split(",")]
    for v in values:                       # warm every variant once
        L.knob_set(a.knob, v)
        trainer.step(pixels, target)
    torch.cuda.synchronize()
    times = {v: [] for v in values}
    for r in range(a.rounds):
        order = values[r % len(values):] + values[:r % len(values)]
        for v in order:
            L.knob_set(a.knob, v)
            trainer.step(pixels, target)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                trainer.step(pixels, target)
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) / a.steps * 1e3)
        print(f"round {r + 1}/{a.rounds}", flush=True)
    out = {"knob": a.knob, "batch": B, "steps": a.steps, "rounds": a.rounds, "variants": {}}
    for v in values:
        L.knob_set(a.knob, v)
        ops.timing_enable((1 << len(L.TIMER_NAMES)) - 1)
        trainer.step(pixels, target)
        torch.cuda.synchronize()
        kern = {}
        for tid, name in enumerate(L.TIMER_NAMES):
            n, ms, work = ops.timing_collect(tid, with_bytes=True)
            if n and (name.startswith("conv") or name == "bn"):
                kern[name] = {"ms": round(ms, 3), "launches": n,
                              **({"tflops": round(work / (ms / 1e3) / 1e12, 2)} if name.startswith("conv") else {})}
        ops.timing_enable(0)
        t = times[v]
        out["variants"][str(v)] = {"ms_per_step_median": round(statistics.median(t), 3), "min": round(min(t), 3),
                                   "max": round(max(t), 3), "clips_per_s": round(B / statistics.median(t) * 1e3, 2),
                                   "kernels": kern}
        print(f"{a.knob}={v}: {json.dumps(out['variants'][str(v)])}", flush=True)
    L.knob_set(a.knob, 0)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
