"""Interleaved A/B of the C3 forward / dX block products over one knob's values, in ONE process
(cdna_hip_programming.md rule 24): rounds x values, each timing `--reps` back-to-back launches of
every product on the same random bf16 operands (rule 25), plus a bitwise comparison of every value's
outputs with the first value's (a schedule-only change must not move a bit).
Usage: python scripts/gemm_c3_ab.py --knob g256_a3 --values 0,1 [--rounds 5 --reps 5 --only fwd]"""
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
    ap.add_argument("--knob", default="g256_a3")
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rows", type=int, default=200704)
    ap.add_argument("--only", default="")
    ap.add_argument("--json", default="")
    ap.add_argument("--dw", action="store_true", help="also time the four dW products")
    a = ap.parse_args()
    M, D, F = a.rows, 768, 3072
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    values = [int(v, 0) for v in a.values.split(",")]

    def rnd(*s, scale=1.0):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(bf)
    prods = {"fwd_qkv": (3 * D, D, L.EPI_BIAS, bf, True),
             "fwd_proj": (D, D, L.EPI_BIAS | L.EPI_RESIDUAL, torch.float32, True),
             "fwd_fc1": (F, D, L.EPI_BIAS | L.EPI_GELU | L.EPI_GELU_GRAD, bf, True),
             "fwd_fc1plain": (F, D, L.EPI_BIAS, bf, True),   # diagnostic: fc1's shape without the GELU epilogue
             "fwd_fc2": (D, F, L.EPI_BIAS | L.EPI_RESIDUAL, torch.float32, True),
             "dx_fc2": (F, D, L.EPI_MUL_AUX, bf, False), "dx_fc1": (D, F, 0, torch.float32, False),
             "dx_proj": (D, D, 0, bf, False), "dx_qkv": (D, 3 * D, 0, torch.float32, False)}
    out = {"knob": a.knob, "values": values, "M": M, "rounds": a.rounds, "reps": a.reps, "products": {}}
    for name, (N, K, epi, odt, bkc) in prods.items():
        if a.only and not name.startswith(a.only):
            continue
        x = rnd(M, K)
        w = rnd(N, K, scale=K ** -0.5)
        wb = w if bkc else w.t().contiguous()
        c = torch.empty(M, N, dtype=odt, device=dev)
        bias = torch.randn(N, device=dev, generator=g)
        res = torch.randn(M, N, device=dev, generator=g) if epi & L.EPI_RESIDUAL else None
        aux_out = torch.empty(M, N, dtype=bf, device=dev) if epi & L.EPI_GELU else None
        aux_in = rnd(M, N) if epi & L.EPI_MUL_AUX else None
        kw = dict(M=M, N=N, K=K, a_kcontig=True, b_kcontig=bkc, lda=K, ldb=K if bkc else N, ldc=N, epilogue=epi,
                  bias=bias if epi & L.EPI_BIAS else None, residual=res, ld_residual=N if res is not None else 0,
                  aux_out=aux_out, ld_aux_out=N if aux_out is not None else 0, aux_in=aux_in,
                  ld_aux_in=N if aux_in is not None else 0)
        ref = None
        same = {}
        paths = {}
        for v in values:
            L.knob_set(a.knob, v)
            c.fill_(7.0)
            L.dispatch_reset()
            ops.gemm(x, wb, c, **kw)
            torch.cuda.synchronize()
            paths[v] = [k for k, n in L.dispatch_counts().items() if n]
            if ref is None:
                ref = c.clone()
            same[v] = bool(torch.equal(c, ref))
        times = {v: [] for v in values}
        for r in range(a.rounds):
            order = values[r % len(values):] + values[:r % len(values)]
            for v in order:
                L.knob_set(a.knob, v)
                ops.gemm(x, wb, c, **kw)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                s.record()
                for _ in range(a.reps):
                    ops.gemm(x, wb, c, **kw)
                e.record()
                torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / a.reps * 1e3)
        fl = 2.0 * M * N * K
        ent = {}
        for v in values:
            med = statistics.median(times[v])
            ent[str(v)] = {"median_us": round(med, 1), "min_us": round(min(times[v]), 1),
                           "frac": round(fl / (med * 1e-6) / PEAK, 4), "bitwise_vs_first": same[v], "path": paths[v]}
        out["products"][name] = ent
        print(f"{name:9s} " + "  ".join(f"{a.knob}={v}: {ent[str(v)]['median_us']:8.1f} us "
                                          f"({ent[str(v)]['frac']:.3f}) {'=' if same[v] else 'DIFF'} {paths[v]}"
                                          for v in values), flush=True)
        del x, w, wb, c, res, aux_out, aux_in, ref
    if a.dw:   # the weight-gradient products (dW = dY^T X over the 200,704 tokens, + bias gradient)
        for name, (Mo, No) in {"dw_qkv": (3 * D, D), "dw_proj": (D, D), "dw_fc1": (F, D), "dw_fc2": (D, F)}.items():
            if a.only and not name.startswith(a.only):
                continue
            dy = rnd(M, Mo)
            xx = rnd(M, No)
            c = torch.zeros(Mo, No, device=dev)
            db = torch.zeros(Mo, device=dev)
            ws = torch.empty(ops.splitk_workspace_bytes(bf, Mo, No, M) // 4 + 64, device=dev)
            times = {v: [] for v in values}
            for r in range(a.rounds):
                order = values[r % len(values):] + values[:r % len(values)]
                for v in order:
                    L.knob_set(a.knob, v)
                    ops.linear_dw(dy, xx, c, db=db, workspace=ws)
                    s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    s0.record()
                    for _ in range(a.reps):
                        ops.linear_dw(dy, xx, c, db=db, workspace=ws)
                    e0.record()
                    torch.cuda.synchronize()
                    times[v].append(s0.elapsed_time(e0) / a.reps * 1e3)
            fl = 2.0 * M * Mo * No
            ent = {str(v): {"median_us": round(statistics.median(times[v]), 1), "min_us": round(min(times[v]), 1),
                            "frac": round(fl / (statistics.median(times[v]) * 1e-6) / PEAK, 4)} for v in values}
            out["products"][name] = ent
            print(f"{name:9s} " + "  ".join(f"{a.knob}={v}: {ent[str(v)]['median_us']:8.1f} us ({ent[str(v)]['frac']:.3f})"
                                              for v in values), flush=True)
            del dy, xx, c, ws
    L.knob_set(a.knob, 0)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
