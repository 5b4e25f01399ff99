"""The host kd-tree build (kdtree.cpp RefKDTree, the reference's nanoflann 1.2.3 divideTree /
middleSplit_ / planeSplit, nanoflann.hpp:1046-1186) node for node against the numpy restatement
in tools/kd_shapes.py: structure, vind, cut dimensions and values, divlow / divhigh, depths and
every point box, on tie-heavy sets (duplicated zero code vectors make the deep chains whose
extremes the build carries from parent to child)."""
import os
import sys

import numpy as np
import pytest

import quant_amd

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import kd_shapes  # noqa: E402

sys.setrecursionlimit(20000)


def _sets():
    rng = np.random.default_rng(11)
    for D in (3, 12, 48):
        for K in (7, 64, 300, 1024):
            for levels in (2, 5, 50, 0):
                P = rng.random((K, D)) if levels == 0 else rng.integers(0, levels, (K, D)) / levels
                P[rng.random(K) < 0.3] = 0.0   # duplicated zero code vectors
                yield "D%d K%d L%d" % (D, K, levels), P
    # a deep chain: most points at zero, the rest spread along a few dimensions each
    P = np.zeros((1024, 48))
    for i in range(1024 - 700):
        P[i, rng.integers(0, 48, 3)] = rng.random(3) * (1 + i % 7)
    yield "chain", P


def _bfs(nodes):
    order = [0]
    for q in order:
        n = nodes[q]
        if not n["leaf"]:
            order += [n["child1"], n["child2"]]
    return order


@pytest.mark.parametrize("name,P", list(_sets()), ids=lambda x: x if isinstance(x, str) else "")
def test_host_build_matches_the_restatement(name, P):
    ref, vind, _ = kd_shapes.build(P)
    nodes, lo, hi, hvind, depth = quant_amd.host_kdtree_image(P)
    np.testing.assert_array_equal(hvind, vind)
    order = _bfs(ref)
    assert len(nodes) == len(order)
    assert depth == max(n["depth"] for n in ref)
    for q, i in enumerate(order):
        r, h = ref[i], nodes[q]
        assert (h["left"], h["right"], h["depth"]) == (r["left"], r["right"], r["depth"]), (name, q)
        assert (h["child1"] < 0) == r["leaf"], (name, q)
        if not r["leaf"]:
            assert h["divfeat"] == r["cutfeat"] and h["cutval"] == r["cutval"], (name, q)
            assert h["divlow"] == r["divlow"] and h["divhigh"] == r["divhigh"], (name, q)
        if r["right"] > r["left"]:
            pts = P[vind[r["left"]:r["right"]]]
            np.testing.assert_array_equal(lo[q], pts.min(0), err_msg="%s node %d" % (name, q))
            np.testing.assert_array_equal(hi[q], pts.max(0), err_msg="%s node %d" % (name, q))
