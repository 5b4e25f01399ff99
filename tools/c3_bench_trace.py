"""C3 quantizes as bench.py times them (no per-level events), for a kernel trace."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import quant_amd  # noqa: E402

eng = quant_amd.Engine(0)
eng.set_synthetic(4096, 0x5EED, 1, 2, 2, quant_amd.SCALED)
eng.set_timing(-2)
out = (np.empty((1024, eng.dim), np.float64), np.zeros(1, np.float64))
for i in range(8):
    t = time.perf_counter()
    eng.lbg(10, want_assign=False, out=out)
    print("quantize %d: %.3f ms" % (i, (time.perf_counter() - t) * 1e3), flush=True)
print("kahan_redo", eng.timings()["kahan_redo"])
