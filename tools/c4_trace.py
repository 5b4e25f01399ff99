"""C4 quantizes as bench.py times them (no per-level events): wall per quantize."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import quant_amd  # noqa: E402

eng = quant_amd.Engine(0)
eng.set_synthetic(4096, 0x5EED, 1, 4, 4, quant_amd.SCALED)
eng.set_timing(-2)
out = (np.empty((4096, eng.dim), np.float64), np.zeros(1, np.float64))
for i in range(5):
    t = time.perf_counter()
    eng.lbg(12, want_assign=False, out=out)
    print("quantize %d: %.3f ms" % (i, (time.perf_counter() - t) * 1e3), flush=True)
tm = eng.timings()
print("kahan_redo", tm["kahan_redo"], "wait", [round(x, 3) for x in tm["wait_ms"]], "tree", [round(x, 3) for x in tm["tree_ms"]])
