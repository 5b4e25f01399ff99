"""Repeated quantizes of one corpus case on one context (with and without a one-rank RCCL
communicator), each against the oracle's Kahan rule: mismatching indices and kahan_redo per call.

    python tools/repeat_diag.py [timing_level]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import quant_amd  # noqa: E402
from oracle import oracle  # noqa: E402
from kahan_fuzz import make_case  # noqa: E402

timing = int(sys.argv[1]) if len(sys.argv) > 1 else -2
corpus = json.load(open(os.path.join(ROOT, "tests", "golden", "kahan_divergent.json")))
cases = [c for c in corpus["found"] if c["kind"] == "palette" and c["seed"] == 213050489] + corpus["found"][:3]
for case in cases:
    rgb = make_case(case["kind"], case["seed"], case["side"])
    side, bw, bh, bits = case["side"], case["bw"], case["bh"], case["bits"]
    X, _ = oracle.tile(rgb, side, side, bw, bh, pad_code=128)
    _, A_k, _ = oracle.lbg(X, bits, sum_mode=0)
    for comm in (False, True):
        with quant_amd.Engine(0) as eng:
            eng.set_timing(timing)
            if comm:
                eng.comm_init(1, 0, quant_amd.Engine.comm_unique_id())
            eng.set_images(rgb, 1, side, side, bw, bh, quant_amd.SCALED)
            out = []
            for rep in range(4):
                C, A, d = eng.lbg(bits)
                out.append((int((A != A_k).sum()), eng.timings()["kahan_redo"]))
        print(case["kind"], case["seed"], "comm" if comm else "plain", "timing", timing, out, flush=True)
