"""rocprofv3 --pmc passes (scripts/pmc_attn.sh) -> per-kernel JSON with derived utilisations.

Per kernel (averaged over its dispatches): every counter, plus
  kernel_cycles   = GRBM_GUI_ACTIVE / 8            (rocprofv3 sums GRBM over the 8 XCDs)
  mfma_busy_frac  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * kernel_cycles)
  wave_cycles     = 4 * SQ_WAVE_CYCLES              (SQ_* cycle counters count quad-cycles)
  active/wait_any/wait_inst fractions of the wave cycles (disjoint, MI355X_MICROARCH.md PMC table)
  lds_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  hbm_bytes       = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes; FETCH doubled per the gfx950 note)
usage: python scripts/pmc_json.py <pmc dir> <out.json> [kernel-name substrings...]"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main(d, out, filt):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if filt and not any(x in name for x in filt):
                continue
            vals[name.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for name, cs in vals.items():
        a = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"counters": a, "dispatches": max(len(v) for v in cs.values())}
        if "GRBM_GUI_ACTIVE" in a:
            kc = a["GRBM_GUI_ACTIVE"] / 8.0
            e["kernel_cycles"] = kc
            if "SQ_VALU_MFMA_BUSY_CYCLES" in a:
                e["mfma_busy_frac"] = a["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * kc)
        if "SQ_WAVE_CYCLES" in a:
            wc = a["SQ_WAVE_CYCLES"]
            for k, c in (("active_frac", "SQ_ACTIVE_INST_ANY"), ("wait_any_frac", "SQ_WAIT_ANY"),
                         ("wait_inst_frac", "SQ_WAIT_INST_ANY")):
                if c in a:
                    e[k] = a[c] / wc
        if a.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_conflict_frac"] = a.get("SQ_LDS_BANK_CONFLICT", 0.0) / a["SQ_LDS_IDX_ACTIVE"]
        if "FETCH_SIZE" in a and "WRITE_SIZE" in a:
            e["hbm_bytes"] = (2 * a["FETCH_SIZE"] + a["WRITE_SIZE"]) * 1024.0
        if "TCC_HIT_sum" in a and "TCC_MISS_sum" in a and a["TCC_HIT_sum"] + a["TCC_MISS_sum"] > 0:
            e["l2_hit_frac"] = a["TCC_HIT_sum"] / (a["TCC_HIT_sum"] + a["TCC_MISS_sum"])
        if "TA_BUSY_avr" in a and "GRBM_GUI_ACTIVE" in a:
            e["ta_busy_frac"] = a["TA_BUSY_avr"] / (a["GRBM_GUI_ACTIVE"] / 8.0)
        if a.get("TCP_TCC_READ_REQ_sum"):
            e["l2_read_latency_cycles"] = a.get("TCP_TCC_READ_REQ_LATENCY_sum", 0.0) / a["TCP_TCC_READ_REQ_sum"]
        res[name] = e
    json.dump({"source": d, "kernels": res}, open(out, "w"), indent=1, sort_keys=True)
    for n, e in res.items():
        print(f"{n[:60]:60s} mfma_busy {e.get('mfma_busy_frac', float('nan')):.3f} "
              f"active {e.get('active_frac', float('nan')):.2f} wait {e.get('wait_any_frac', float('nan')):.2f} "
              f"stall {e.get('wait_inst_frac', float('nan')):.2f} l2hit {e.get('l2_hit_frac', float('nan')):.2f} "
              f"ta {e.get('ta_busy_frac', float('nan')):.2f} l2lat {e.get('l2_read_latency_cycles', float('nan')):.0f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
