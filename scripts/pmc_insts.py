"""Per-kernel sums of the SQ counters of one rocprofv3 --pmc pass (any counter
names): python scripts/pmc_insts.py <dir> [kernel substring]"""
import csv
import glob
import sys
from collections import defaultdict

base = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(float))
nd = defaultdict(set)
for f in glob.glob(f"{base}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if sub and sub not in k:
            continue
        acc[k[:60]][r["Counter_Name"]] += float(r["Counter_Value"])
        nd[k[:60]].add(r.get("Dispatch_Id", ""))
for k, v in sorted(acc.items()):
    print(k, "dispatches", len(nd[k]))
    for c, x in sorted(v.items()):
        print(f"   {c:24s} {x:16.0f}")
