"""The device build of the reference kd-tree (k_kdbuild.hip) against the host's RefKDTree, node
for node: vind order, cut dimension and value, divlow / divhigh, the split records the tie
certificate replays (candidate dimensions, clamp midpoint, spread gap), every node's point box,
the root box and the depth (nanoflann.hpp:1046-1186 via kdtree.cpp; the host tree itself is
checked against the reference's own nanoflann in tests/test_oracle_golden.py).  Cases: the split
codebook of every level of C2 (512^2, 2x2, 10 bits) and of the Kahan corpus (oracle splits), of a
4x4 12-bit run (the engine's splits: C4's degenerate trees, depth 174 at K = 4096), and tie-heavy
random sets of every size class."""
import json
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle

pytestmark = pytest.mark.gpu


def _check(engine, C, what):
    res, ms, why = engine.kdtree_device_check(C)
    assert res == 0, "%s (K=%d, D=%d): %s" % (what, C.shape[0], C.shape[1], why or "device build gave up")
    return ms


def test_random_tie_heavy_sets(engine):
    rng = np.random.default_rng(11)
    for K, D in [(1, 3), (5, 12), (10, 1), (11, 2), (12, 12), (100, 5), (129, 48), (777, 12), (1500, 64),
                 (4096, 48), (4096, 12), (2048, 3)]:
        for levels in (3, 50, 1000):   # few distinct values: ties everywhere; then near-distinct
            C = rng.integers(0, levels, (K, D)).astype(np.float64) / levels
            C[rng.random(K) < 0.2] = 0.0          # duplicated zero rows (empty cells)
            _check(engine, C, "random levels=%d" % levels)
    C = np.full((300, 12), 0.25)                   # every point equal
    _check(engine, C, "all equal")


def test_c2_and_corpus_level_trees(engine):
    X, _ = oracle.tile(oracle.gen_image(512, 0x5EED), 512, 512, 2, 2)
    _, _, _, splits, _ = oracle.lbg(X, 10, sum_mode=0, dump=True)
    for L, C in enumerate(splits):
        _check(engine, C, "C2 level %d" % (L + 1))
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "helpers"))
    from kahan_env_worker import make
    corpus = json.load(open(os.path.join(GOLDEN, "kahan_divergent.json")))
    for c in corpus["noise_seeds"] + corpus["found"]:
        X, _ = oracle.tile(make(c), c["side"], c["side"], c["bw"], c["bh"])
        _, _, _, splits, _ = oracle.lbg(X, c["bits"], sum_mode=0, dump=True)
        for L, C in enumerate(splits):
            _check(engine, C, "corpus %s level %d" % (c, L + 1))


def test_c4_level_trees(engine):
    """A 4096^2 4x4 run's split codebooks (the engine's: lbg with 1..11 levels, then x1.2 | x0.8),
    K = 4 ... 4096 at D = 48: the degenerate trees of duplicate zero code vectors."""
    import quant_amd
    engine.set_synthetic(4096, 0x5EED, 1, 4, 4, quant_amd.SCALED)
    times = {}
    for L in range(1, 12):
        C, _, _ = engine.lbg(L, want_assign=False)
        S = np.concatenate([C * (1 + 0.2), C * (1 - 0.2)])
        times[S.shape[0]] = _check(engine, S, "C4 level %d" % (L + 1))
    print("device build ms by K:", times)


def test_lbg_device_and_host_trees_agree(engine, tmp_path):
    """qvq_lbg with the device trees (QVQ_KDTREE=device, its own process: the switch is read once;
    48-D levels from K = 512) and with host trees (the default) return the same codebook, indices
    and distortion on a 4x4 12-bit run of a 1024^2 image."""
    import subprocess
    import quant_amd
    engine.set_synthetic(1024, 0x5EED, 1, 4, 4, quant_amd.SCALED)
    C, A, d = engine.lbg(12)
    out = str(tmp_path / "device.npz")
    code = ("import sys, numpy as np; sys.path.insert(0, %r); import quant_amd\n"
            "e = quant_amd.Engine(0); e.set_synthetic(1024, 0x5EED, 1, 4, 4, quant_amd.SCALED)\n"
            "C, A, d = e.lbg(12); np.savez(%r, C=C, A=A, d=np.array([d]))\n" %
            (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), out))
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, QVQ_KDTREE="device"),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    h = np.load(out)
    np.testing.assert_array_equal(h["A"], A)
    np.testing.assert_array_equal(h["C"], C)
    assert float(h["d"][0]) == d
