"""Per-level kernel time of the last quantize in a rocprofv3 kernel trace, every kernel counted
(the levels split at each search launch), plus the quantize's span (first kernel start to last end).

    python tools/level_view.py TRACE.csv [--names]
"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = max(i for i, r in enumerate(rows) if "mean_sums" in r["Kernel_Name"])
    rows = rows[last:]
    # the quantize ends at the next mean_sums (none: the end of the trace)
    levels, cur, names = [], defaultdict(float), defaultdict(float)
    levels.append(cur)
    for r in rows:
        n = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "assign_" in n:
            cur = defaultdict(float)
            levels.append(cur)
        key = n.split("(")[0].split("<")[0].replace("void ", "").replace("qvq::", "").replace("(anonymous namespace)::", "")
        cur[key] += d
        names[key] += d
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    busy = sum(names.values())
    for i, L in enumerate(levels):
        print("%3d %8.1f  %s" % (i, sum(L.values()), " ".join("%s=%.1f" % (k, v) for k, v in sorted(L.items(), key=lambda kv: -kv[1]))
                                  if "--names" in sys.argv else ""))
    print("busy %.1f us, span %.1f us" % (busy, span))
    for k, v in sorted(names.items(), key=lambda kv: -kv[1]):
        print("  %-40s %8.1f" % (k[:40], v))


if __name__ == "__main__":
    main()
