"""Interleaved A/B of attention kernel variants in ONE process (cdna_hip_programming.md rule 24):
R rounds x V variants (VS_KNOB_ATTN_VARIANT values), each round times every variant's forward and
backward over `--reps` back-to-back launches on the same random data (rule 25: q, k, v ~ N(0, s^2));
reports per variant the median and min over rounds, the fraction of the 2.5 PF bf16 roof (forward
4 B H N^2 64 FLOP; backward 2.5x that, the credited convention), and whether every variant's outputs
are bitwise equal to the first variant's (the pipelined orders compute the same MFMA chains in the
same order, so they must be).

usage: python scripts/attn_ab.py --variants 0,7 [--batch 128 --heads 3 --rounds 7 --reps 10]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from vspike import _lib as L, ops  # noqa: E402

PEAK = 2.5e15


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,7")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--heads", type=int, default=3)
    ap.add_argument("--tokens", type=int, default=1568)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--only", default="", help="fwd | bwd")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    B, N, H = a.batch, a.tokens, a.heads
    M, Da = B * N, H * 64
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(7)
    qkv = (torch.randn(M, 3 * Da, device=dev, generator=g) * a.scale).to(torch.bfloat16)
    do = (torch.randn(M, Da, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    o = torch.empty(M, Da, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B, H, N, device=dev)
    dq = torch.empty(M, 3 * Da, dtype=torch.bfloat16, device=dev)
    ws = torch.empty(ops.attn_bwd_workspace_bytes(B, N, H) // 4 + 64, device=dev)
    variants = [int(t, 0) for t in a.variants.split(",")]
    fl_f = 4.0 * B * H * N * N * 64
    fl_b = 2.5 * fl_f
    ref_o = ref_lse = ref_dq = None
    same = {}
    for v in variants:     # correctness vs the first variant (and the forward's output feeds the backward)
        L.knob_set("attn_variant", v)
        ops.attn_fwd(qkv, o, lse, B, N, H)
        ops.attn_bwd(qkv, o, do, lse, dq, ws, B, N, H)
        torch.cuda.synchronize()
        if ref_o is None:
            ref_o, ref_lse, ref_dq = o.clone(), lse.clone(), dq.clone()
        same[v] = {"fwd_bitwise": bool(torch.equal(o, ref_o) and torch.equal(lse, ref_lse)),
                   "bwd_bitwise": bool(torch.equal(dq, ref_dq)),
                   "o_maxdiff": float((o.float() - ref_o.float()).abs().max()),
                   "dq_maxdiff": float((dq.float() - ref_dq.float()).abs().max())}
    # the backward runs on the first variant's forward outputs in every round
    o.copy_(ref_o)
    lse.copy_(ref_lse)
    times = {v: {"fwd": [], "bwd": []} for v in variants}

    def timed(fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(a.reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.reps * 1e3
    o2 = torch.empty_like(o)
    lse2 = torch.empty_like(lse)
    for r in range(a.rounds):
        order = variants[r % len(variants):] + variants[:r % len(variants)]
        for v in order:
            L.knob_set("attn_variant", v)
            if a.only != "bwd":
                times[v]["fwd"].append(timed(lambda: ops.attn_fwd(qkv, o2, lse2, B, N, H)))
            if a.only != "fwd":
                times[v]["bwd"].append(timed(lambda: ops.attn_bwd(qkv, o, do, lse, dq, ws, B, N, H)))
        print(f"round {r + 1}/{a.rounds}", flush=True)
    L.knob_set("attn_variant", 0)
    out = {"B": B, "N": N, "H": H, "reps": a.reps, "rounds": a.rounds, "scale": a.scale, "variants": {}}
    for v in variants:
        ent = {"check": same[v]}
        for k, fl in (("fwd", fl_f), ("bwd", fl_b)):
            t = times[v][k]
            if not t:
                continue
            med = statistics.median(t)
            ent[k] = {"median_us": round(med, 1), "min_us": round(min(t), 1), "max_us": round(max(t), 1),
                      "frac_median": round(fl / (med * 1e-6) / PEAK, 4)}
        out["variants"][f"{v:#x}"] = ent
        print(f"variant {v:#x}: {json.dumps(ent)}")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
