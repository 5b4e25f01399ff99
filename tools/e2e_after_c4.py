"""Diagnostics: end-to-end compress timing after a C4 quantize on the same engine (bench.py's
order), split into set_images / lbg."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import quant_amd
from bench import synthetic_raster

S = 4096
eng = quant_amd.Engine(0)
if len(sys.argv) > 1 and sys.argv[1] == "c4":
    eng.set_synthetic(S, 0x5EED, 1, 4, 4, quant_amd.SCALED)
    eng.lbg(12, want_assign=False)
rgb = synthetic_raster(S, 0x5EED)
C = np.empty((1024, 12), np.float64)
d = np.zeros(1, np.float64)
parts = {"set": [], "lbg": []}
for r in range(6):
    t0 = time.perf_counter()
    eng.set_images(rgb, 1, S, S, 2, 2, quant_amd.SCALED)
    t1 = time.perf_counter()
    eng.lbg(10, out=(C, d))
    t2 = time.perf_counter()
    parts["set"].append(round((t1 - t0) * 1e3, 3))
    parts["lbg"].append(round((t2 - t1) * 1e3, 3))
print(json.dumps({"after": sys.argv[1:] or ["none"], **parts}))
