"""GPU parity on inputs where the reference's Kahan centroid bits decide an index.

The reference sums each centroid with Kahan's compensation in ascending row order
(src/Quantizer.cpp:59-70); the engine's exact sums can differ from it by an ulp, and on the
inputs here that ulp changes which code vector a near-tied row gets (oracle sum_mode 0 vs 1
disagree).  The engine must return the Kahan rule's indices: levels whose recheck leaves rows
in the tie band recompute the previous level's centroids with the reference's bits
(k_kahan.hip) before the kd-tree answers them.

Corpus: the verdict's four noise seeds and the cases tools/kahan_fuzz.py found
(tests/golden/kahan_divergent.json: generator parameters only; the oracle recomputes the
expected indices here)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle

pytestmark = pytest.mark.gpu

CORPUS = json.load(open(os.path.join(GOLDEN, "kahan_divergent.json")))


def _make(case):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(GOLDEN), "..", "tools"))
    if case["kind"] == "noise96":
        return np.random.default_rng(case["seed"]).integers(0, 256, 96 * 96 * 3, dtype=np.uint8)
    from kahan_fuzz import make_case
    return make_case(case["kind"], case["seed"], case["side"])


def _check(engine, case, cs=oracle.SCALED):
    rgb = _make(case)
    side, bw, bh, bits = case["side"], case["bw"], case["bh"], case["bits"]
    X, _ = oracle.tile(rgb, side, side, bw, bh, cs=cs, pad_code=128 if cs == oracle.SCALED else 0)
    C_k, A_k, d_k = oracle.lbg(X, bits, sum_mode=0)
    _, A_x, _ = oracle.lbg(X, bits, sum_mode=1)
    engine.set_images(rgb, 1, side, side, bw, bh, cs)
    C, A, d = engine.lbg(bits)
    np.testing.assert_array_equal(A, A_k)     # the reference's rule
    # the engine's codebook is the exact-sum centroid of its (the reference's) final cells
    np.testing.assert_array_equal(C, oracle.centroids(X, A_k, 1 << bits, sum_mode=1))
    assert np.max(np.abs(C - C_k) / np.maximum(np.abs(C_k), 1e-300)) <= 1e-12
    assert abs(d - d_k) <= 1e-9 * abs(d_k)
    return int((A_k != A_x).sum())


@pytest.mark.parametrize("case", CORPUS["noise_seeds"], ids=lambda c: f"noise96-seed{c['seed']}")
def test_noise_seeds_follow_the_kahan_rule(engine, case):
    assert _check(engine, case) > 0   # the exact-sum rule differs here


@pytest.mark.parametrize("case", CORPUS["found"],
                         ids=lambda c: f"{c['kind']}-{c['seed']}-{c['side']}-{c['bw']}x{c['bh']}-n{c['bits']}")
def test_fuzz_corpus_follows_the_kahan_rule(engine, case):
    assert _check(engine, case) > 0


def test_normal_colour_space_needs_no_kahan(engine):
    # NORMAL values are integers: the Kahan sums are exact, both rules agree
    case = dict(kind="noise96", seed=26, side=96, bw=2, bh=2, bits=10)
    assert _check(engine, case, cs=oracle.NORMAL) == 0
