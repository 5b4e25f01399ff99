"""Find inputs on which the reference's Kahan centroid rule and the exact-sum rule give
different codebook indices (oracle only, CPU).  Writes tests/golden/kahan_divergent.json: the
generator parameters of every divergent case, the corpus the GPU tests replay
(tests/test_gpu_kahan.py) against the Kahan oracle.

    python tools/kahan_fuzz.py [cases] [seed0]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402

KINDS = ("noise", "palette", "gen", "flat", "saturated", "dark")


def make_case(kind, seed, side):
    """A side x side raster of one kind (deterministic in seed)."""
    rng = np.random.default_rng(seed)
    n = side * side * 3
    if kind == "noise":
        return rng.integers(0, 256, n, dtype=np.uint8)
    if kind == "palette":
        pal = rng.integers(0, 256, (int(rng.integers(2, 9)), 3), dtype=np.uint8)
        return pal[rng.integers(0, len(pal), side * side)].reshape(-1)
    if kind == "gen":
        return oracle.gen_image(side, seed=int(seed))[: n]
    if kind == "flat":
        base = rng.integers(0, 256, 3)
        noise = rng.integers(-2, 3, (side * side, 3))
        return np.clip(base + noise, 0, 255).astype(np.uint8).reshape(-1)
    if kind == "saturated":
        v = rng.integers(0, 256, n)
        v[rng.random(n) < 0.4] = 255
        return v.astype(np.uint8)
    if kind == "dark":
        return rng.integers(0, 12, n, dtype=np.uint8)
    raise ValueError(kind)


def run_case(kind, seed, side, bw, bh, bits):
    rgb = make_case(kind, seed, side)
    X, _ = oracle.tile(rgb, side, side, bw, bh)
    _, A0, _ = oracle.lbg(X, bits, sum_mode=0)
    _, A1, _ = oracle.lbg(X, bits, sum_mode=1)
    return int((A0 != A1).sum())


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rng = np.random.default_rng(seed0)
    found = []
    for i in range(cases):
        kind = KINDS[i % len(KINDS)]
        seed = int(rng.integers(0, 1 << 30))
        side = int(rng.choice([32, 48, 64, 96]))
        bw, bh = int(rng.integers(1, 5)), int(rng.integers(1, 4))
        bits = int(rng.integers(3, 11))
        nd = run_case(kind, seed, side, bw, bh, bits)
        if nd:
            found.append(dict(kind=kind, seed=seed, side=side, bw=bw, bh=bh, bits=bits, rows=nd))
            print(found[-1], flush=True)
    out = dict(cases=cases, seed0=seed0, divergent=len(found), rate=len(found) / cases, found=found,
               noise_seeds=[dict(kind="noise96", seed=s, side=96, bw=2, bh=2, bits=10) for s in (26, 109, 203, 356)])
    path = os.path.join(ROOT, "tests", "golden", "kahan_divergent.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(found)} of {cases} cases diverge; wrote {path}")


if __name__ == "__main__":
    main()
