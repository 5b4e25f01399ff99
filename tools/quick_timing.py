"""Per-level timings of qvq_lbg for a few workloads (diagnostics, not the bench)."""
import json
import sys
import time

sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import quant_amd

cases = [(512, 2, 10), (4096, 2, 10), (4096, 4, 12)]
if len(sys.argv) > 1:
    cases = [tuple(int(v) for v in c.split(',')) for c in sys.argv[1:]]
eng = quant_amd.Engine(0)
# per-level events (off by default: each record idles the GPU ~6 us, so a kernel trace taken with
# them shows ~6 us gaps around every search); QT_EVENTS=0 leaves them off (the schedule as bench.py
# runs it; the per-level times then read 0)
eng.set_timing(-2 if __import__('os').environ.get("QT_EVENTS") == "0" else -1)
for (S, bw, bits) in cases:
    eng.set_synthetic(S, 0x5EED, 1, bw, bw)
    for rep in range(3):
        t = time.time()
        C, A, d = eng.lbg(bits, want_assign=False)
        dt = time.time() - t
    tm = eng.timings()
    print(json.dumps({"S": S, "bw": bw, "bits": bits, "wall_ms": round(dt * 1e3, 3), "total_ms": round(tm["total_ms"], 3),
                      "assign_ms": [round(x, 4) for x in tm["assign_ms"]],
                      "update_ms": [round(x, 4) for x in tm["update_ms"]],
                      "other_ms": [round(x, 4) for x in tm["other_ms"]],
                      "flagged": tm["flagged"], "host_ties": tm["host_ties"],
                      "wait_ms": [round(x, 3) for x in tm["wait_ms"]], "tree_ms": [round(x, 3) for x in tm["tree_ms"]]}),
          flush=True)
