"""Diagnostic: one corpus case through a no-communicator and a one-rank-communicator engine:
indices vs the oracle's Kahan rule, kahan_redo, per-level ties."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "helpers"))
import numpy as np  # noqa: E402
import quant_amd  # noqa: E402
from oracle import oracle  # noqa: E402
from kahan_env_worker import make  # noqa: E402

case = json.loads(sys.argv[1]) if len(sys.argv) > 1 else dict(kind="noise96", seed=26, side=96, bw=2, bh=2, bits=10)
rgb = make(case)
X, _ = oracle.tile(rgb, case["side"], case["side"], case["bw"], case["bh"])
_, A_k, _, sp, asg = oracle.lbg(X, case["bits"], sum_mode=0, dump=True)
_, A_x, _ = oracle.lbg(X, case["bits"], sum_mode=1)
for comm in (False, True):
    eng = quant_amd.Engine(0)
    if comm:
        eng.comm_init(1, 0, quant_amd.Engine.comm_unique_id())
    eng.set_images(rgb, 1, case["side"], case["side"], case["bw"], case["bh"])
    C, A, d = eng.lbg(case["bits"])
    tm = eng.timings()
    bad = np.nonzero(A != A_k)[0]
    print("comm", comm, "mismatch", len(bad), "rows", bad[:8].tolist(), "eng", A[bad[:8]].tolist(), "ref", A_k[bad[:8]].tolist(),
          "exact", A_x[bad[:8]].tolist(), "redo", tm["kahan_redo"], "ties", tm["host_ties"], flush=True)
    eng.close()
