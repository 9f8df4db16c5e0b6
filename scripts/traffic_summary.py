"""Per-kernel HBM bytes per launch from the two rocprofv3 --pmc passes of scripts/pmc_traffic.sh.
traffic = 2 * FETCH_SIZE + WRITE_SIZE (rocprofv3 reports KB; gfx950 FETCH_SIZE counts half of a
wide streaming read, MI355X_MICROARCH.md "HBM").  Also groups the attention backward op
(row prep + dK/dV + dQ kernels) the way bench.py's roofline counts it."""
import csv
import glob
import json
import sys
from collections import defaultdict


def main(d, out, steps):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    kern = {}
    for name, c in vals.items():
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        fetch = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
        write = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
        kern[name.split("(")[0]] = {"fetch_bytes_x2": 2 * fetch, "write_bytes": write, "traffic_bytes": 2 * fetch + write,
                                    "launches": len(c["FETCH_SIZE"])}
    # the bench's timer classes (libvspike VS_TIMER_*): which kernels one timed call launches
    groups = {"attn_bwd": ["attn_rowprep_kernel", "attn_bwd_bf16_kernel", "attn_bwd_bf16_pp_kernel", "attn_bwd_dkdv_bf16_kernel",
                           "attn_bwd_dq_bf16_kernel"],
              "attn_fwd": ["attn_fwd_bf16_kernel"],
              "gemm_dw": ["gemm_dw_kernel", "gemm_dw_reg_kernel", "gemm_dw_reduce"],
              "gemm": ["gemm_bf16_kernel", "gemm_bf16_ring_kernel", "gemm_bf16_fullk_kernel", "gemm_bf16_panel_kernel",
                       "gemm_f32_kernel", "gemm_skinny_kernel", "gemm_splitk_reduce"],
              "ln_fwd": ["ln_fwd_vec_kernel", "ln_fwd_kernel"],
              "ln_bwd": ["ln_bwd_vec_kernel", "ln_bwd_kernel", "ln_partsum_kernel"],
              "adamw": ["adamw_kernel"]}
    grouped = {}
    for g, parts in groups.items():
        hit = [k for k in kern if any(k.split("<")[0].endswith(p) for p in parts)]
        if hit:
            # per timed call: launches of a class can differ per kernel (a reduce after a split-K
            # kernel), so the class total per step is divided by its anchor kernel's launch count
            anchor = max(hit, key=lambda k: kern[k]["traffic_bytes"] * kern[k]["launches"])
            tot = sum(kern[k]["traffic_bytes"] * kern[k]["launches"] for k in hit)
            grouped[g] = {"traffic_bytes": tot / kern[anchor]["launches"], "kernels": hit,
                          "bytes_per_step": tot / steps, "anchor": anchor}
    json.dump({"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, bench.py --steps 3 --warmup 1; "
                         "traffic = 2*FETCH_SIZE + WRITE_SIZE per launch (bytes); ops: per bench timer class, "
                         "bytes_per_step = class bytes over the profiled run / train steps in it",
               "steps": steps,
               "ops": grouped, "kernels": kern}, open(out, "w"), indent=1, sort_keys=True)
    for g, v in grouped.items():
        print(g, f"{v['traffic_bytes'] / 1e6:.1f} MB/launch")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 4)
