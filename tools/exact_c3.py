"""Exact mode on C3-sized CIE1931 data: the reference's generic quantize (include/Quantizer.hpp:10-16)
on the 2x2 blocks of the S x S synthetic raster mapped through CIE1931 (src/ColorSpace.cpp:30-38),
which only the exact mode (k_exact.hip) takes.  Prints one JSON line: wall ms per quantize and the
engine's per-phase timings.

  python3 tools/exact_c3.py [--side 4096] [--bits 10] [--reps 2] [--check-side 0]

--check-side S2 > 0 also runs the oracle (sum_mode=0, the reference's Kahan rule) on an S2 x S2 image
and asserts indices and codebook bit-equal (test infrastructure only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=4096)
    ap.add_argument("--bits", type=int, default=10)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--check-side", type=int, default=0)
    a = ap.parse_args()
    import quant_amd
    from bench import cie_blocks, synthetic_raster
    eng = quant_amd.Engine(0)
    if a.check_side:
        from oracle import oracle
        s = a.check_side
        X = cie_blocks(synthetic_raster(s, 7), s)
        Xr, _ = oracle.tile(synthetic_raster(s, 7), s, s, 2, 2, cs=oracle.NORMAL)
        p = Xr.reshape(-1, 3)
        ref = np.stack([(p[:, 0] * 0.490 + p[:, 1] * 0.310 + p[:, 2] * 0.200) / 0.17697,
                        (p[:, 0] * 0.17697 + p[:, 1] * 0.81240 + p[:, 2] * 0.01063) / 0.17697,
                        (p[:, 0] * 0 + p[:, 1] * 0.01 + p[:, 2] * 0.99) / 0.17697], axis=1).reshape(-1, 12)
        assert np.array_equal(X, ref), "block layout differs from the oracle's tiling"
        C_r, A_r, _ = oracle.lbg(X, a.bits, sum_mode=0, threads=8)
        eng.set_vectors(X, exact=True)
        C, A, _ = eng.lbg(a.bits)
        assert np.array_equal(A, A_r) and np.array_equal(C, C_r), "exact mode differs from the oracle"
        print("check %dx%d bits %d: indices and codebook bit-equal to the oracle" % (s, s, a.bits), flush=True)
    X = cie_blocks(synthetic_raster(a.side, 7), a.side)
    t0 = time.perf_counter()
    eng.set_vectors(X, exact=True)
    set_ms = (time.perf_counter() - t0) * 1e3
    eng.lbg(a.bits)   # warm-up (allocations)
    ms = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        eng.lbg(a.bits)
        ms.append((time.perf_counter() - t0) * 1e3)
    tm = eng.timings()
    print(json.dumps({"workload": "C3 CIE1931 exact", "side": a.side, "rows": int(X.shape[0]), "dim": 12,
                      "bits": a.bits, "ms": [round(v, 2) for v in ms], "best_ms": round(min(ms), 2),
                      "set_vectors_ms": round(set_ms, 1), "ties": tm["host_ties"],
                      "assign_ms": [round(v, 2) for v in tm["assign_ms"]],
                      "update_ms": [round(v, 2) for v in tm["update_ms"]]}), flush=True)


if __name__ == "__main__":
    main()
