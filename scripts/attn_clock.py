"""Effective clock and matrix-pipe occupancy of the attention kernels in one rocprofv3 run
(--pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES with --kernel-trace): per dispatch, clock =
(GRBM_GUI_ACTIVE / 8 XCDs) / duration, MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM/8);
the executed busy x clock / 2.4 GHz is the roof fraction the matrix pipe alone would give.
usage: python scripts/attn_clock.py <rocprofv3 output dir> [kernel substring ...] [--json out.json]"""
import csv
import glob
import sys
from collections import defaultdict


def main(d, filt):
    trace = {}
    for f in glob.glob(f"{d}/*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            trace[r["Dispatch_Id"]] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    cnt = defaultdict(dict)
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            cnt[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    per = defaultdict(list)
    for did, cs in cnt.items():
        if did not in trace or "GRBM_GUI_ACTIVE" not in cs:
            continue
        name, ns = trace[did]
        if filt and not any(x in name for x in filt):
            continue
        cyc = cs["GRBM_GUI_ACTIVE"] / 8.0
        per[name.split("(")[0]].append((ns, cyc, cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024.0 * cyc)))
    print(f"{'kernel':60s} {'calls':>5s} {'us':>9s} {'GHz':>6s} {'mfma_busy':>9s} {'busy x clk/2.4':>14s}")
    res = {}
    for n, v in sorted(per.items()):
        us = sum(x[0] for x in v) / len(v) / 1e3
        ghz = sum(x[1] / x[0] for x in v) / len(v)
        busy = sum(x[2] for x in v) / len(v)
        res[n] = {"us": round(us, 1), "clock_ghz": round(ghz, 3), "mfma_busy_frac": round(busy, 4),
                  "busy_x_clock_frac": round(busy * ghz / 2.4, 4), "calls": len(v)}
        print(f"{n[:60]:60s} {len(v):5d} {us:9.1f} {ghz:6.3f} {busy:9.3f} {busy * ghz / 2.4:14.3f}")
    return res


if __name__ == "__main__":
    args = sys.argv[2:]
    out = None
    if "--json" in args:
        i = args.index("--json")
        out = args[i + 1]
        args = args[:i] + args[i + 2:]
    r = main(sys.argv[1], args)
    if out:
        import json
        json.dump({"source": sys.argv[1], "kernels": r}, open(out, "w"), indent=1, sort_keys=True)
