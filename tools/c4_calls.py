"""Wall time of consecutive qvq_lbg calls on one workload (default C4: 4096^2, 4x4 blocks, 12
bits), no timing events: median / min / max over the calls after 3 warmup calls.
usage: python tools/c4_calls.py [S,bw,bits] [calls]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import quant_amd  # noqa: E402

S, bw, bits = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "4096,4,12").split(","))
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 40
eng = quant_amd.Engine(0)
eng.set_timing(-2)
eng.set_synthetic(S, 0x5EED, 1, bw, bw)

t = []
for i in range(calls + 3):
    t0 = time.perf_counter()
    eng.lbg(bits, want_assign=False)
    if i >= 3:
        t.append((time.perf_counter() - t0) * 1e3)
t.sort()
print(json.dumps({"case": [S, bw, bits], "calls": calls, "median_ms": round(t[len(t) // 2], 3), "min_ms": round(t[0], 3),
                  "p90_ms": round(t[int(len(t) * 0.9)], 3)}))
