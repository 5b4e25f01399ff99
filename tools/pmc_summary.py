"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_summary.py OUT.json FETCH_DIR WRITE_DIR [WORKLOAD_KEY]

FETCH_SIZE / WRITE_SIZE are in KB per dispatch.  MI355X_MICROARCH.md (HBM section): on
gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so fetch bytes are
doubled; WRITE_SIZE is taken as is.  Kernel names are shortened to the qvq:: name.
"""
import csv
import glob
import json
import os
import re
import sys


def short(name):
    m = re.search(r"qvq(?:::|\d+)([A-Za-z_]+?)(?:_kernel)?(?:I|E|\(|$)", name)
    m3 = re.search(r"assign_small_kernel(?:ILi(\d+)ELb([01])E|<(\d+), (true|false)[,>])", name)
    if m3:
        sk = m3.group(1) or m3.group(3)
        fused = m3.group(2) == "1" or m3.group(4) == "true"
        return "assign_small_kernel<%s,%s>" % (sk, "fused" if fused else "plain")
    m4 = re.search(r"assign_mf32_kernelILb([01])ELb([01])ELi(\d+)ELb([01])ELb([01])E", name)
    if m4:
        return "assign_mf32_kernel<%s,%s,U%s%s%s>" % ("fused" if m4.group(1) == "1" else "plain",
                                                     "staged" if m4.group(2) == "1" else "global", m4.group(3),
                                                     ",tag" if m4.group(4) == "1" else "",
                                                     ",prune" if m4.group(5) == "1" else "")
    m2 = re.search(r"assign_mfma_kernelILb([01])ELb([01])E", name)
    if m2:
        return "assign_mfma_kernel<%s,%s>" % ("fused" if m2.group(1) == "1" else "plain",
                                              "staged" if m2.group(2) == "1" else "global")
    for key in ["mean_sums_kernel", "finalize_prep_kernel", "recheck_mf32_kernel", "recheck_kernel",
                "decode_rows_h_kernel", "decode_rows_kernel", "decode_pixels_kernel", "kd_resolve_kernel", "kd_reduce_kernel",
                "reduce_kernel",
                "update_kernel", "assign_valu_kernel", "tile_kernel", "gen_kernel", "byte_hist_kernel",
                "prep_kernel", "copyBuffer", "fillBuffer"]:
        if key in name:
            return key
    return m.group(1) if m else name[:60]


def load(d, counter):
    out = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") != counter:
                continue
            k = short(r["Kernel_Name"])
            out.setdefault(k, []).append(float(r["Counter_Value"]))
    return out


def main():
    out, fdir, wdir = sys.argv[1:4]
    workload = sys.argv[4] if len(sys.argv) > 4 else None
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    res = {"note": "bytes per launch; fetch = 2 x FETCH_SIZE (gfx950 correction), write = WRITE_SIZE",
           "workload": workload, "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        fb = 2 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        res["kernels"][k] = {"launches": max(len(f), len(w)),
                             "fetch_bytes": round(fb) if fb is not None else None,
                             "write_bytes": round(wb) if wb is not None else None,
                             "hbm_bytes": round((fb or 0) + (wb or 0))}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
