"""Debug: one corpus case on the engine (env selects the path) against the oracle's two rules."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: F401,E402
import quant_amd  # noqa: E402
from oracle import oracle  # noqa: E402

cs = int(sys.argv[1]) if len(sys.argv) > 1 else 0
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 26
bits = int(sys.argv[3]) if len(sys.argv) > 3 else 10
rgb = np.random.default_rng(seed).integers(0, 256, 96 * 96 * 3, dtype=np.uint8)
X, _ = oracle.tile(rgb, 96, 96, 2, 2, cs=cs, pad_code=128 if cs == oracle.SCALED else 0)
eng = quant_amd.Engine(0)
for b in range(1, bits + 1):
    _, A_k, _ = oracle.lbg(X, b, sum_mode=0)
    _, A_x, _ = oracle.lbg(X, b, sum_mode=1)
    eng.set_images(rgb, 1, 96, 96, 2, 2, cs)
    C, A, d = eng.lbg(b)
    t = eng.timings()
    print(f"cs {cs} bits {b}: A!=A_k {(A != A_k).sum()}  A!=A_x {(A != A_x).sum()}  A_k!=A_x {(A_k != A_x).sum()} ties {t['host_ties'][b-1]}",
          flush=True)
