"""Per-quantize GPU busy vs wall from a rocprofv3 kernel trace: the span from each
mean_sums_kernel to the following copy_out_kernel, the sum of kernel durations inside it, and
the idle gaps larger than a threshold (host-side stalls)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
spans = []
cur = None
for r in rows:
    n = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if "mean_sums_kernel" in n:
        cur = {"t0": s, "busy": 0, "prev_end": s, "gaps": []}
    if cur is None:
        continue
    g = (s - cur["prev_end"]) / 1e3
    if g > thr:
        cur["gaps"].append((round(g, 1), n.split("(")[0][-30:]))
    cur["busy"] += e - s
    cur["prev_end"] = e
    if "copy_out_kernel" in n:
        spans.append(((e - cur["t0"]) / 1e3, cur["busy"] / 1e3, cur["gaps"]))
        cur = None
for w, b, g in spans[-6:]:
    print("wall %7.1f us  busy %7.1f us  idle %6.1f us  gaps>%g: %s" % (w, b, w - b, thr, g))
