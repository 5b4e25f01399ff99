"""Levels of a reference run for tests/cpp/test_tie_cert.cpp: per level the exact-sum split (the
exact centroids of the reference's previous assignment, split), the reference's Kahan-bit split,
the tie band's rows (in_tie_band over the exact split's best two distances, common.hpp) plus a
few ordinary rows, and the reference's indices for them.

  python3 tools/tie_cert_data.py SIDE BW BH BITS OUT [extra_rows]   (the synthetic image)
  python3 tools/tie_cert_data.py --corpus OUT                          (the Kahan corpus)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import oracle  # noqa: E402


def ref_l2(X, C):
    """kdtree_dev.hpp ref_l2_hd for every (row, code vector) pair: [n, K] (same IEEE order)."""
    n, D = X.shape
    r = np.zeros((n, C.shape[0]))
    d = 0
    while d + 3 < D:
        e = [X[:, None, d + i] - C[None, :, d + i] for i in range(4)]
        r += (e[1] * e[1] + e[2] * e[2]) + (e[0] * e[0] + e[3] * e[3])
        d += 4
    while d < D:
        e = X[:, None, d] - C[None, :, d]
        r += e * e
        d += 1
    return r


def band_rows(X, C, tie_abs, chunk=1 << 15):
    import torch
    Xt = torch.from_numpy(X)
    Ct = torch.from_numpy(C)
    cn = (Ct * Ct).sum(1)
    out = []
    for s in range(0, X.shape[0], chunk):
        xb = Xt[s:s + chunk]
        dd = (xb * xb).sum(1)[:, None] - 2 * xb @ Ct.T + cn[None, :]
        top = torch.topk(dd, 2, dim=1, largest=False).values if C.shape[0] > 1 else None
        if top is None:
            continue
        near = (top[:, 1] - top[:, 0] <= 1e-9).nonzero().flatten().numpy() + s
        if len(near) == 0:
            continue
        p = np.sort(ref_l2(X[near], C), axis=1)
        d1, d2 = p[:, 0], p[:, 1]
        band = tie_abs * (np.sqrt(d1) + np.sqrt(np.minimum(d2, 1e300))) + tie_abs * tie_abs
        keep = (d2 - d1 <= 1e-12 * d1) | (d2 - d1 <= band)
        out.append(near[keep])
    return np.concatenate(out) if out else np.zeros(0, np.int64)


def write_levels(f, X, bits, extra, rng):
    N, D = X.shape
    tie_abs = 2 * 2.0 ** -49 * np.sqrt(D)
    _, _, _, splits, assigns = oracle.lbg(X, bits, sum_mode=0, threads=8, dump=True)
    counts = []
    for lvl in range(1, bits + 1):
        K = 1 << lvl
        A_prev = assigns[lvl - 2] if lvl > 1 else np.zeros(N, np.uint32)
        cent = oracle.centroids(X, A_prev, K // 2, sum_mode=1)
        ex = np.concatenate([cent * (1 + 0.2), cent * (1 - 0.2)])
        rows = band_rows(X, ex, tie_abs)
        rows = np.unique(np.concatenate([rows, rng.integers(0, N, extra)]))
        f.write(np.array([K, D, len(rows)], np.uint32).tobytes())
        f.write(np.ascontiguousarray(ex).tobytes())
        f.write(np.ascontiguousarray(splits[lvl - 1]).tobytes())
        f.write(np.ascontiguousarray(X[rows]).tobytes())
        f.write(assigns[lvl - 1][rows].astype(np.uint32).tobytes())
        counts.append(len(rows))
    return counts


def corpus_cases():
    """The Kahan corpus (tests/golden/kahan_divergent.json) as (name, X, bits)."""
    import json
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from kahan_fuzz import make_case
    c = json.load(open(os.path.join(here, "..", "tests", "golden", "kahan_divergent.json")))
    for case in c["noise_seeds"] + c["found"]:
        side = case["side"]
        if case["kind"] == "noise96":
            rgb = np.random.default_rng(case["seed"]).integers(0, 256, side * side * 3, dtype=np.uint8)
        else:
            rgb = make_case(case["kind"], case["seed"], side)
        X, _ = oracle.tile(rgb, side, side, case["bw"], case["bh"], pad_code=128)
        yield "%s-%d" % (case["kind"], case["seed"]), X, case["bits"]


def main():
    rng = np.random.default_rng(5)
    if sys.argv[1] == "--corpus":
        with open(sys.argv[2], "wb") as f:
            for name, X, bits in corpus_cases():
                print(name, "rows per level", write_levels(f, X, bits, 20, rng), flush=True)
        return
    side, bw, bh, bits = (int(v) for v in sys.argv[1:5])
    out = sys.argv[5]
    extra = int(sys.argv[6]) if len(sys.argv) > 6 else 200
    X, _ = oracle.tile(oracle.gen_image(side), side, side, bw, bh)
    with open(out, "wb") as f:
        print("rows per level", write_levels(f, X, bits, extra, rng))


if __name__ == "__main__":
    main()
