"""Exact mode (VERDICT r02 missing #2): the AbstractQuantizer path accepts any training set, as the
reference's `quantize(const std::vector<Vector>&, n, eps)` does (include/Quantizer.hpp:10-16).
Values that are not byte images of a colour space -- random doubles, CIE1931-like values, other
dimensions -- go through qvq_set_vectors' exact mode: fp64 search in nanoflann's order with
kd-tree ties (src/Quantizer.cpp:24-32), Kahan sums of each cell's rows in ascending order times
fl(1/n) (src/Quantizer.cpp:46-87).  The bar is bit-identity with the oracle's Kahan rule
(oracle.lbg(sum_mode=0), the reference's arithmetic): indices AND codebook; the distortion (an
OpenMP reduction in the reference, order-dependent in its last bits) within 1e-12 relative.
Byte-image data can be forced through the same mode (exact=True) and then also matches the
reference's Kahan codebook bit for bit, where the fast path's exact sums are within 1 ulp."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _check(engine, X, bits, exact=False):
    C_r, A_r, d_r = oracle.lbg(X, bits, sum_mode=0)
    engine.set_vectors(X, exact=exact)
    C, A, d = engine.lbg(bits)
    np.testing.assert_array_equal(A, A_r)
    np.testing.assert_array_equal(C, C_r)
    assert abs(d - d_r) <= 1e-12 * abs(d_r)
    return C, A


@pytest.mark.parametrize("D,N,bits", [(12, 6000, 7), (3, 5000, 6), (48, 1500, 5), (1, 777, 4), (20, 333, 9)])
def test_random_fp64_data(engine, D, N, bits):
    rng = np.random.default_rng(D * 1000 + N)
    X = rng.normal(size=(N, D)) * rng.uniform(0.1, 10, size=D) + rng.uniform(-5, 5, size=D)
    _check(engine, X, bits)


def test_cie_like_values(engine):
    """The reference's CIE1931 map (src/ColorSpace.cpp:30-38) applied to every pixel of the 2x2
    blocks: values off the 2^-60 grid, so only the exact mode can take them."""
    X, _ = oracle.tile(oracle.gen_image(64, 0x5EED), 64, 64, 2, 2, cs=oracle.NORMAL)   # signed chars
    p = X.reshape(-1, 3)
    xyz = np.stack([(p[:, 0] * 0.490 + p[:, 1] * 0.310 + p[:, 2] * 0.200) / 0.17697,
                    (p[:, 0] * 0.17697 + p[:, 1] * 0.81240 + p[:, 2] * 0.01063) / 0.17697,
                    (p[:, 0] * 0 + p[:, 1] * 0.01 + p[:, 2] * 0.99) / 0.17697], axis=1)
    _check(engine, xyz.reshape(-1, 12), 8)


def test_duplicates_and_ties(engine):
    """Repeated rows, repeated code vectors (zero rows split to equal code vectors) and exact
    distance ties: the kd-tree's first-visited rule decides, as in the reference."""
    rng = np.random.default_rng(5)
    base = rng.integers(0, 4, size=(40, 6)).astype(np.float64) * 0.25
    X = np.concatenate([base[rng.integers(0, 40, size=3000)], np.zeros((200, 6))])
    _check(engine, X, 7)


def test_byte_data_forced_exact_matches_kahan_bits(engine):
    """beans-like byte data through the exact mode: the Kahan codebook bit for bit (the fast path
    agrees with it to <= 1 ulp and on every index)."""
    X, _ = oracle.tile(oracle.gen_image(128, 0x5EED), 128, 128, 2, 2)
    C_e, A_e = _check(engine, X, 8, exact=True)
    engine.set_vectors(X)
    C_f, A_f, _ = engine.lbg(8)
    np.testing.assert_array_equal(A_f, A_e)
    np.testing.assert_allclose(C_f, C_e, rtol=4e-16, atol=0)


def test_single_steps(engine):
    """qvq_assign / qvq_update in exact mode: the oracle's kd-tree answer and Kahan centroids."""
    rng = np.random.default_rng(11)
    X = rng.normal(size=(4000, 12))
    C = rng.normal(size=(37, 12))
    engine.set_vectors(X)
    A = engine.assign(C)
    np.testing.assert_array_equal(A, oracle.kdtree_nn(C, X))
    C2, cnt = engine.update(A, 37)
    np.testing.assert_array_equal(C2, oracle.centroids(X, A, 37, sum_mode=0))
    np.testing.assert_array_equal(cnt, np.bincount(A, minlength=37))


def test_lbg_quantizer_plugin_generic(engine):
    """getQuantizer(LBG).quantize on arbitrary vectors (the drop-in's generic callers)."""
    import quant_amd
    rng = np.random.default_rng(2)
    X = rng.uniform(-1, 1, size=(2000, 4))
    C, A, d = quant_amd.getQuantizer(quant_amd.Quantizers.LBG).quantize(X, 5, 1e-6)
    C_r, A_r, d_r = oracle.lbg(X, 5, sum_mode=0)
    np.testing.assert_array_equal(A, A_r)
    np.testing.assert_array_equal(C, C_r)
