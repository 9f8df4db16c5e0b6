"""Average rocprofv3 --pmc counter values per kernel (name substring filter) across passes."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
filt = sys.argv[2:] or [""]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{d}/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in vals.items():
    if not any(x in name for x in filt):
        continue
    print(name[:90])
    for c, v in sorted(cs.items()):
        print(f"   {c:32s} {sum(v)/len(v):16.1f}  (n={len(v)})")
