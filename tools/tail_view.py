"""The end of the last quantize in a rocprofv3 kernel trace: every kernel from the last level's
search launch on, with its start relative to that launch, its duration and its queue (the main
stream's and the check's side stream's kernels apart), plus the span to the trace's last kernel.

    python tools/tail_view.py TRACE.csv [levels_back]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    search = [i for i, r in enumerate(rows) if "assign_" in r["Kernel_Name"]]
    i0 = search[-back]
    t0 = int(rows[i0]["Start_Timestamp"])
    qcol = next((c for c in ("Queue_Id", "Stream_Id", "Queue_ID") if c in rows[0]), None)
    for r in rows[i0:]:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("qvq::", "").replace("(anonymous namespace)::", "")
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print("%9.1f %8.1f  q%-3s %s" % ((s - t0) / 1e3, (e - s) / 1e3, r.get(qcol, "?") if qcol else "?", n[:70]))
    print("span from the level's search to the last kernel's end: %.1f us" % ((int(rows[-1]["End_Timestamp"]) - t0) / 1e3))


if __name__ == "__main__":
    main()
