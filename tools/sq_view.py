"""Per-launch SQ counters (tools/gpu_pmc_sq.sh output) for the last quantize's kernels."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 10
vals = defaultdict(dict)
names = {}
for path in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        key = (path.split("/p")[1].split("/")[0], int(r["Dispatch_Id"]))
        vals[key][r["Counter_Name"]] = vals[key].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
        names[key] = r["Kernel_Name"]
by_pass = defaultdict(list)
for (p, disp), v in sorted(vals.items()):
    if sys.argv[3] if len(sys.argv) > 3 else "assign" in names[(p, disp)]:
        by_pass[p].append(v)
cols = {}
for p, lst in by_pass.items():
    for i, v in enumerate(lst[-last:]):
        cols.setdefault(i, {}).update(v)
keys = sorted({k for v in cols.values() for k in v})
for k in keys:
    print("%-28s" % k, " ".join("%10.3g" % cols[i].get(k, float("nan")) for i in sorted(cols)))
