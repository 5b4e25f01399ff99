"""Host-side logic of the product (no GPU): C-ABI exports, the host kd-tree resolver,
the exact-sum finaliser, and the fail-loudly behaviour without a device."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from oracle import oracle


def test_library_exports_every_declared_symbol():
    import quant_amd
    L = quant_amd.lib()
    hdr = open(os.path.join(ROOT, "include", "qvq.h")).read()
    names = re.findall(r"QVQ_API\s+[\w\s\*]+?\b(qvq_\w+)\s*\(", hdr)
    assert len(names) >= 18
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(quant_amd.EXPORTED)


def test_no_device_fails_loudly():
    import torch
    import quant_amd
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(quant_amd.QVQError):
        quant_amd.Engine(0)


def test_host_kdtree_matches_oracle():
    import quant_amd
    rng = np.random.default_rng(5)
    X, _ = oracle.tile(oracle.gen_image(96), 96, 96, 2, 2)
    for K in (1, 2, 11, 100, 513):
        base = X[rng.choice(len(X), K, replace=False)]
        C = np.concatenate([base * (1 + 0.2), base * (1 - 0.2), np.zeros((2, 12))])
        np.testing.assert_array_equal(quant_amd.host_kdtree_nn(C, X), oracle.kdtree_nn(C, X))
    # 4x4 blocks (D = 48) and 1x1 (D = 3: leftover-component path of the distance)
    for bw in (1, 4):
        X, _ = oracle.tile(oracle.gen_image(64), 64, 64, bw, bw)
        C = np.concatenate([X[:50] * 1.2, X[:50] * 0.8, X[:5]])
        np.testing.assert_array_equal(quant_amd.host_kdtree_nn(C, X), oracle.kdtree_nn(C, X))
    # bigger D = 48 trees (C4-sized codebooks)
    X, _ = oracle.tile(oracle.gen_image(192), 192, 192, 4, 4)
    for K in (1100, 3000):
        base = X[rng.choice(len(X), K // 2, replace=False)]
        C = np.concatenate([base * (1 + 0.2), base * (1 - 0.2), np.zeros((2, 48))])
        np.testing.assert_array_equal(quant_amd.host_kdtree_nn(C, X), oracle.kdtree_nn(C, X))


@pytest.mark.parametrize("cs", [oracle.SCALED, oracle.NORMAL])
def test_exact_sum_finaliser(cs):
    import quant_amd
    X, codes = oracle.tile(oracle.gen_image(128), 128, 128, 2, 2, cs=cs, pad_code=128 if cs else 0)
    rng = np.random.default_rng(1)
    K = 64
    A = rng.integers(0, K - 4, len(X)).astype(np.uint32)
    hi, lo = quant_amd.host_row_terms(codes, cs)
    H = np.zeros((K, 12), np.uint64)
    Lo = np.zeros((K, 12), np.uint64)
    np.add.at(H, A, hi)
    np.add.at(Lo, A, lo)
    cnt = np.bincount(A, minlength=K).astype(np.uint64)
    C = quant_amd.host_finalize(H, Lo, cnt, cs)
    np.testing.assert_array_equal(C, oracle.centroids(X, A, K, sum_mode=1))


@pytest.mark.parametrize("scenario,status,max_s", [
    (0, 0, 0.15),     # the work publishes after ~5 ms
    (1, 3, 1.0),      # never publishes, no communicator: QVQ_EDEVICE at the timeout
    (2, 4, 1.0),      # never publishes, communicator joined: QVQ_ECOMM (a peer rank stalled)
    (3, 4, 0.15),     # the communicator reports a peer failure: QVQ_ECOMM before the timeout
    (4, 3, 0.15),     # the stream faults: QVQ_EDEVICE
    (5, 3, 0.15),     # the stream drains without publishing: QVQ_EDEVICE
])
def test_bounded_wait_policy(scenario, status, max_s):
    """Every host wait of the engine on its stream is bounded (failure
    detection): a dead peer rank or a faulted stream ends the call with a status instead of
    hanging (quant_amd/csrc/wait.hpp, exercised through qvq_host_wait_probe)."""
    import quant_amd
    st, el = quant_amd.host_wait_probe(scenario, 0.25)
    assert st == status
    assert el <= max_s
    if scenario in (1, 2):
        assert el >= 0.25



def test_bench_cie_blocks_follow_the_reference_tiling():
    """bench.py's exact_cie1931 input: getBlocksAsVectorsFromImage (the oracle's NORMAL tiling,
    src/Compressor.cpp:31-62) of the synthetic raster, each pixel through CIE1931
    (src/ColorSpace.cpp:30-38)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    S = 64
    rgb = bench.synthetic_raster(S, 0x5EED)
    X = bench.cie_blocks(rgb, S)
    Xr, _ = oracle.tile(rgb, S, S, 2, 2, cs=oracle.NORMAL)
    p = Xr.reshape(-1, 3)
    ref = np.stack([(p[:, 0] * 0.490 + p[:, 1] * 0.310 + p[:, 2] * 0.200) / 0.17697,
                    (p[:, 0] * 0.17697 + p[:, 1] * 0.81240 + p[:, 2] * 0.01063) / 0.17697,
                    (p[:, 0] * 0 + p[:, 1] * 0.01 + p[:, 2] * 0.99) / 0.17697], axis=1).reshape(-1, 12)
    np.testing.assert_array_equal(X, ref)


def test_cert_pool_runs_each_slot_once():
    """pool_run's helpers read a job's epoch, width and fn together, and a helper
    spawned later starts from the current epoch -- no slot runs twice or is skipped while the
    width grows and shrinks from job to job."""
    import quant_amd
    assert quant_amd.host_pool_stress(3000, 13) == 0
    assert quant_amd.host_pool_stress(300, 64) == 0
