"""Kernel timeline from a rocprofv3 kernel trace.

    python tools/trace_view.py TRACE.csv [N]            last N kernels: start, duration, gap
    python tools/trace_view.py TRACE.csv --compact      per-level table of the last quantize
"""
import csv
import sys

SHORT = [("assign_small", "search"), ("assign_mfma", "search"), ("assign_mf32", "search"), ("assign_wide", "search"),
         ("assign_valu", "search"), ("recheck", "recheck"), ("kd_resolve", "kd"), ("reduce_kernel", "reduce"),
         ("finalize_prep", "final"), ("finalize_kernel", "final"), ("reduce_split", "final"), ("update_runs", "update")]


def short(name):
    for key, s in SHORT:
        if key in name:
            return s
    return None


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if "--compact" not in sys.argv:
        n = int(sys.argv[2]) if len(sys.argv) > 2 else 80
        rows = rows[-n:]
        t0 = int(rows[0]["Start_Timestamp"])
        prev_end = t0
        for r in rows:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            name = r["Kernel_Name"]
            name = name if len(name) < 70 else name[:70]
            print("%9.1f us  dur %7.1f  gap %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev_end) / 1e3, name))
            prev_end = e
        return
    last = max(i for i, r in enumerate(rows) if "mean_sums" in r["Kernel_Name"])
    levels, cur = [], None
    for r in rows[last:]:
        k = short(r["Kernel_Name"])
        if k is None:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if k == "search":
            cur = {}
            levels.append(cur)
        if cur is not None:
            cur[k] = cur.get(k, 0.0) + d
    cols = ["search", "recheck", "kd", "update", "reduce", "final"]
    print("lvl " + " ".join("%8s" % c for c in cols))
    tot = {c: 0.0 for c in cols}
    for i, L in enumerate(levels):
        print("%3d " % (i + 1) + " ".join("%8.1f" % L.get(c, 0.0) for c in cols))
        for c in cols:
            tot[c] += L.get(c, 0.0)
    print("sum " + " ".join("%8.1f" % tot[c] for c in cols) + "   all %.1f us" % sum(tot.values()))


if __name__ == "__main__":
    main()
