"""Interleaved A/B of the LayerNorm backward over one knob's values in ONE process (rule 24), at a
bench geometry (default C3: 200,704 rows x 768, bf16 dy, f32 x / residual gradient, f32 + bf16 dx),
plus a bitwise check of every value's dx / dgamma against the first value's.
usage: python scripts/ln_ab.py --knob ln_blocks --values 0,768,512 [--rows 200704 --cols 768]"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))

import torch  # noqa: E402

from vspike import _lib as L, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", default="ln_blocks")
    ap.add_argument("--values", default="0,768,512")
    ap.add_argument("--rows", type=int, default=200704)
    ap.add_argument("--cols", type=int, default=768)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--json", default="")
    ap.add_argument("--fwd", action="store_true", help="time the forward (x f32 -> y bf16, mean, rstd) instead")
    a = ap.parse_args()
    R, C = a.rows, a.cols
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    dy = torch.randn(R, C, device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn(R, C, device=dev, generator=g)
    mean = x.mean(1)
    rstd = torch.rsqrt(x.var(1, unbiased=False) + 1e-12)
    gamma = torch.randn(C, device=dev, generator=g)
    dres = torch.randn(R, C, device=dev, generator=g)
    dx = torch.empty(R, C, device=dev)
    dx_lp = torch.empty(R, C, dtype=torch.bfloat16, device=dev)
    dg = torch.zeros(C, device=dev)
    db = torch.zeros(C, device=dev)
    ws = torch.empty(ops.layernorm_bwd_workspace_bytes(R, C) // 4 + 4, device=dev)
    values = [int(v, 0) for v in a.values.split(",")]

    beta = torch.randn(C, device=dev, generator=g)
    y = torch.empty(R, C, dtype=torch.bfloat16, device=dev)
    mo = torch.empty(R, device=dev)
    ro = torch.empty(R, device=dev)

    def run():
        if a.fwd:
            ops.layernorm_fwd(x, gamma, beta, 1e-12, y, mo, ro)
        else:
            ops.layernorm_bwd(dy, x, mean, rstd, gamma, dx, dg, db, dres=dres, dx_lp=dx_lp, workspace=ws)
    if a.fwd:
        dx, dg = y, mo   # the bitwise check compares the forward's outputs
    ref = None
    same = {}
    for v in values:
        L.knob_set(a.knob, v)
        dg.zero_()
        db.zero_()
        run()
        torch.cuda.synchronize()
        if ref is None:
            ref = (dx.clone(), dg.clone())
        same[v] = bool(torch.equal(dx, ref[0])) and bool(torch.equal(dg, ref[1]))
    times = {v: [] for v in values}
    for r in range(a.rounds):
        order = values[r % len(values):] + values[:r % len(values)]
        for v in order:
            L.knob_set(a.knob, v)
            run()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(a.reps):
                run()
            e.record()
            torch.cuda.synchronize()
            times[v].append(s.elapsed_time(e) / a.reps * 1e3)
    L.knob_set(a.knob, 0)
    nbytes = R * C * (4 + 2) + R * 8 if a.fwd else R * C * (2 + 4 + 4 + 4 + 2)
    out = {"knob": a.knob, "rows": R, "cols": C, "bytes_per_launch": nbytes, "values": {}}
    for v in values:
        med = statistics.median(times[v])
        out["values"][str(v)] = {"median_us": round(med, 1), "min_us": round(min(times[v]), 1),
                                 "tb_s": round(nbytes / (med * 1e-6) / 1e12, 2), "bitwise_vs_first": same[v]}
        print(f"{a.knob}={v}: {json.dumps(out['values'][str(v)])}", flush=True)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
