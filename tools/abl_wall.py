"""Unprofiled host wall per C3 quantize (median of 30) -- compare QVQ_* ablation settings
without the kernel-trace profiler in the loop.  usage: python tools/abl_wall.py [S,bw,bits]"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import quant_amd  # noqa: E402

S, bw, bits = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "4096,2,10").split(","))
eng = quant_amd.Engine(0)
eng.set_synthetic(S, 0x5EED, 1, bw, bw)
eng.set_timing(-2)
ts = []
for rep in range(35):
    t = time.perf_counter()
    eng.lbg(bits, want_assign=False)
    ts.append(time.perf_counter() - t)
ts = ts[5:]
print(json.dumps({"abl": os.environ.get("QVQ_ABL_SKIP", "0"), "S": S, "bits": bits,
                  "median_ms": round(statistics.median(ts) * 1e3, 4), "min_ms": round(min(ts) * 1e3, 4)}), flush=True)
