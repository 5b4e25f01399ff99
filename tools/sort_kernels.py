"""Per-quantize totals of the sort-path kernels in ab_env.sh traces (the last quantize's 8
levels).  usage: python tools/sort_kernels.py NAME..."""
import collections
import csv
import sys

for n in sys.argv[1:]:
    rows = list(csv.DictReader(open("gpurun_out/abe/%s/t_kernel_trace.csv" % n)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    agg = collections.defaultdict(list)
    for r in rows:
        nm = r["Kernel_Name"]
        if "sort" in nm or "fill" in nm:
            agg[nm.split("(")[0].replace("void ", "")[:34]].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    print(n, {k: round(sum(v[-8:]), 1) for k, v in agg.items()})
