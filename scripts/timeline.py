"""Per-step timeline summary from a rocprofv3 --kernel-trace CSV: step span, per-stream busy time,
gaps, and the top kernels by time on each stream (last N steps; a step starts at the im2col kernel).
usage: python scripts/timeline.py <kernel_trace.csv> [steps]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
want = int(sys.argv[2]) if len(sys.argv) > 2 else 3
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
starts = [i for i, r in enumerate(rows) if "im2col" in r["Kernel_Name"] or "patch_embed_fwd" in r["Kernel_Name"]]
starts = starts[-want:]
def short(n):
    n = re.sub(r"\(.*", "", n)
    return n[:70]
for si, i0 in enumerate(starts):
    i1 = starts[si + 1] if si + 1 < len(starts) else len(rows)
    ks = rows[i0:i1]
    t0, t1 = ks[0]["s"], max(k["e"] for k in ks)
    by_q = defaultdict(list)
    for k in ks:
        by_q[k["Queue_Id"]].append(k)
    print(f"step {si}: span {(t1 - t0) / 1e3:.1f} us, {len(ks)} kernels")
    # union of busy intervals over all queues
    iv = sorted((k["s"], k["e"]) for k in ks)
    busy, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f"   any-kernel busy {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us")
    for q, kq in by_q.items():
        tot = sum(k["e"] - k["s"] for k in kq)
        agg = defaultdict(lambda: [0, 0])
        for k in kq:
            a = agg[short(k["Kernel_Name"])]
            a[0] += k["e"] - k["s"]
            a[1] += 1
        top = sorted(agg.items(), key=lambda x: -x[1][0])[:8]
        print(f"   queue {q}: {len(kq)} kernels, busy {tot / 1e3:.1f} us")
        if si == len(starts) - 1:
            for n, (t, c) in top:
                print(f"      {t / 1e3:8.1f} us  x{c:3d}  {n}")
    if True:
        # largest idle gaps of the union timeline, with the kernels on either side
        gaps = []
        end, last = ks[0]["e"], ks[0]
        for k in sorted(ks, key=lambda r: r["s"])[1:]:
            if k["s"] > end:
                gaps.append((k["s"] - end, short(last["Kernel_Name"]), short(k["Kernel_Name"])))
            if k["e"] > end:
                end, last = k["e"], k
        print("   largest idle gaps:")
        for g, a, b in sorted(gaps, reverse=True)[:10]:
            print(f"      {g / 1e3:7.1f} us  after {a[:45]:45s} before {b[:45]}")
