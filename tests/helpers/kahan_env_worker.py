"""Runs corpus cases through one engine in a process whose environment selects a Kahan schedule
(tests/test_gpu_kahan.py: QVQ_SPECULATE=0, QVQ_KAHAN_FAIL_LEVEL, QVQ_KAHAN_DIRECT_MAX; the engine
 reads these once),
printing one JSON line per case: indices and codebook against the oracle's Kahan rule (the
reference's, src/Quantizer.cpp:59-87), a second quantize on the same context, kahan_redo.

    python kahan_env_worker.py '[{"kind": ..., "seed": ..., "side": ..., "bw": ..., "bh": ..., "bits": ...}, ...]'
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def make(case):
    from oracle import oracle
    if case["kind"] == "noise96":
        return np.random.default_rng(case["seed"]).integers(0, 256, 96 * 96 * 3, dtype=np.uint8)
    if case["kind"] == "gen" and case["side"] >= 128:
        return oracle.gen_image(case["side"], seed=int(case["seed"]))
    from kahan_fuzz import make_case
    return make_case(case["kind"], case["seed"], case["side"])


def main():
    import quant_amd
    from oracle import oracle
    cases = json.loads(sys.argv[1])
    eng = quant_amd.Engine(0)
    for case in cases:
        rgb = make(case)
        side, bw, bh, bits = case["side"], case["bw"], case["bh"], case["bits"]
        X, _ = oracle.tile(rgb, side, side, bw, bh)
        _, A_k, _ = oracle.lbg(X, bits, sum_mode=0)
        eng.set_images(rgb, 1, side, side, bw, bh, quant_amd.SCALED)
        C, A, d = eng.lbg(bits)
        redo = eng.timings()["kahan_redo"]
        C2, A2, d2 = eng.lbg(bits)
        print(json.dumps({"case": case, "A_ok": bool(np.array_equal(A, A_k)),
                          "C_ok": bool(np.array_equal(C, oracle.centroids(X, A_k, 1 << bits, sum_mode=1))),
                          "again_ok": bool(np.array_equal(A2, A) and np.array_equal(C2, C) and d2 == d),
                          "redo": redo}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
