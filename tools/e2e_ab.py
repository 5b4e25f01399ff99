"""End-to-end compress timing (host raster -> qvq_set_images -> qvq_lbg -> indices on the host),
the drop-in's PCIe-inclusive region (src/Compressor.cpp:118-123); run under QVQ_H2D=pageable
for the A/B.  Diagnostics, not the bench."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import quant_amd
from bench import synthetic_raster

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
rgb = synthetic_raster(S, 0x5EED)
eng = quant_amd.Engine(0)
C = np.empty((1024, 12), np.float64)
d = np.zeros(1, np.float64)
parts = {"set": [], "lbg": [], "total": []}
for r in range(7):
    t0 = time.perf_counter()
    eng.set_images(rgb, 1, S, S, 2, 2)
    t1 = time.perf_counter()
    _, A, _ = eng.lbg(10, out=(C, d))
    t2 = time.perf_counter()
    if r >= 2:
        parts["set"].append(t1 - t0)
        parts["lbg"].append(t2 - t1)
        parts["total"].append(t2 - t0)
print(json.dumps({"mode": os.environ.get("QVQ_H2D", "register"),
                  **{k: round(sorted(v)[len(v) // 2] * 1e3, 3) for k, v in parts.items()}}))
