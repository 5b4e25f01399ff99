"""GPU parity: the HIP engine against the oracle (lbg_oracle.c) on the same inputs.

Bar: code-vector indices bit-exact; codebooks bit-exact against the oracle's exact-sum
mode (the engine's documented centroid rule) and within 1e-12 relative of the oracle's
Kahan mode (the reference's own rule; north-star tolerance is 1e-5)."""
import numpy as np
import pytest

from conftest import load_png_rgb, reference_lbg
from oracle import oracle

pytestmark = pytest.mark.gpu

KAHAN_RTOL = 1e-12


def _check_against_oracle(engine, rgb, xs, ys, bw, bh, bits, cs=oracle.SCALED):
    import quant_amd
    X, _ = oracle.tile(rgb, xs, ys, bw, bh, cs=cs, pad_code=128 if cs == oracle.SCALED else 0)
    C_e, A_k, d_k, C_k = reference_lbg(X, bits)
    engine.set_images(rgb, 1, xs, ys, bw, bh, cs)
    C, A, d = engine.lbg(bits)
    assert A.shape == A_k.shape
    np.testing.assert_array_equal(A, A_k)          # reference rule (Kahan centroid bits)
    np.testing.assert_array_equal(C, C_e)          # engine centroid rule on those cells, bit-exact
    scale = np.maximum(np.abs(C_k), 1e-300)
    assert np.max(np.abs(C - C_k) / scale) <= KAHAN_RTOL
    assert abs(d - d_k) <= 1e-9 * abs(d_k)
    return C, A, d


def test_beans_n8(engine):
    rgb, xs, ys = load_png_rgb("beans.png")
    _check_against_oracle(engine, rgb, xs, ys, 2, 2, 8)


def test_kodim01_n10(engine):
    rgb, xs, ys = load_png_rgb("kodim01.png")
    _check_against_oracle(engine, rgb, xs, ys, 2, 2, 10)


def test_t_wrap_pad_n4(engine):
    # 510 x 383: odd height exercises the column wrap and the end-of-buffer zero pad.
    rgb, xs, ys = load_png_rgb("t.png")
    _check_against_oracle(engine, rgb, xs, ys, 2, 2, 4)


def test_s512_n10(engine):
    _check_against_oracle(engine, oracle.gen_image(512), 512, 512, 2, 2, 10)


def test_repeated_calls_and_edge_levels(engine):
    # consecutive quantizes on one context: the per-call state (mean buffer the K=1 finalize
    # clears, counters the mean kernel clears, the A memset only bits == 0 needs, the
    # completion flag of the result copy) must not leak from one call into the next
    rgb = oracle.gen_image(128)
    for bits in (6, 0, 1, 0, 5):
        _check_against_oracle(engine, rgb, 128, 128, 2, 2, bits)


@pytest.mark.parametrize("bw,bh,bits", [(1, 1, 5), (1, 3, 6), (2, 4, 6), (4, 4, 8), (3, 3, 7)])
def test_block_shapes(engine, bw, bh, bits):
    _check_against_oracle(engine, oracle.gen_image(96), 96, 96, bw, bh, bits)


def test_normal_colorspace(engine):
    _check_against_oracle(engine, oracle.gen_image(64), 64, 64, 2, 2, 6, cs=oracle.NORMAL)


def test_synthetic_generator_matches(engine):
    rgb = oracle.gen_image(256, 0x5EED + 3)
    engine.set_images(rgb, 1, 256, 256, 2, 2)
    C1, A1, d1 = engine.lbg(7)
    engine.set_synthetic(256, 0x5EED + 3, 1, 2, 2)
    C2, A2, d2 = engine.lbg(7)
    np.testing.assert_array_equal(A1, A2)
    np.testing.assert_array_equal(C1, C2)


def test_multi_image_batch(engine):
    # image-major concatenation (SURVEY.md 8(d) C5 definition) on a small batch
    imgs = [oracle.gen_image(64, 0x5EED + b) for b in range(3)]
    X = np.concatenate([oracle.tile(im, 64, 64, 2, 2)[0] for im in imgs])
    C_e, A_k, _, _ = reference_lbg(X, 6)
    engine.set_synthetic(64, 0x5EED, 3, 2, 2)
    C, A, _ = engine.lbg(6)
    np.testing.assert_array_equal(A, A_k)
    np.testing.assert_array_equal(C, C_e)


def test_set_vectors_path(engine):
    X, _ = oracle.tile(oracle.gen_image(64), 64, 64, 2, 2)
    C_e, A_k, _, _ = reference_lbg(X, 5)
    engine.set_vectors(X)
    C, A, _ = engine.lbg(5)
    np.testing.assert_array_equal(A, A_k)
    np.testing.assert_array_equal(C, C_e)


def test_set_vectors_rejects_bad_data(engine):
    """Non-finite values have no reference answer to match (the exact mode, which takes any other
    data, is tests/test_gpu_exact.py)."""
    import quant_amd
    X = np.random.rand(100, 12)
    X[5, 3] = np.nan
    with pytest.raises(quant_amd.QVQError):
        engine.set_vectors(X)


@pytest.fixture(params=["device", "host"])
def kdmode(request, monkeypatch):
    """Exact fp64 ties go through the device kd-tree traversal (default) or, with
    QVQ_KDTREE=host, the synchronous host resolution; both must give the reference answer."""
    if request.param == "host":
        monkeypatch.setenv("QVQ_KDTREE", "host")
    else:
        monkeypatch.delenv("QVQ_KDTREE", raising=False)
    return request.param


def test_assign_ties_and_duplicates(engine, kdmode):
    """Duplicated code vectors and split pairs (the structural tie sources) are resolved
    exactly as the reference kd-tree resolves them."""
    rng = np.random.default_rng(7)
    X, _ = oracle.tile(oracle.gen_image(128), 128, 128, 2, 2)
    engine.set_vectors(X)
    base = X[rng.choice(len(X), 40, replace=False)]
    C = np.concatenate([base * (1 + 0.2), base * (1 - 0.2), np.zeros((8, 12)), base[:4], base[:4]])
    A = engine.assign(C)
    np.testing.assert_array_equal(A, oracle.kdtree_nn(C, X))
    t = engine.timings()
    assert t["host_ties"][0] > 0      # rows equal to base[:4] tie between the two copies


@pytest.mark.parametrize("bw,bh", [(2, 2), (4, 4)])
def test_kd_tie_sets_across_leaves(engine, bw, bh):
    """Rows with many exactly equidistant code vectors spread over several kd-tree leaves
    (x +- 2^-12 along every component: the differences, hence the distances, are exact),
    next to 100 duplicate zero code vectors (a deep tree) and scaled rows.  The device
    answers such ties from the path order of the tied points (kd_tie_direct), falling back
    to the walk; both must pick the reference kd-tree's first-visited point."""
    rng = np.random.default_rng(19)
    X, _ = oracle.tile(oracle.gen_image(128), 128, 128, bw, bh)
    D = X.shape[1]
    engine.set_vectors(X)
    centres = X[rng.choice(len(X), 24, replace=False)]
    v = 2.0 ** -12
    star = np.concatenate([np.concatenate([c + v * np.eye(D), c - v * np.eye(D)]) for c in centres])
    others = X[rng.choice(len(X), 200, replace=False)] * 0.9
    C = np.concatenate([others[:100], star, np.zeros((100, D)), others[100:]])
    C = C[rng.permutation(len(C))]
    A = engine.assign(C)
    np.testing.assert_array_equal(A, oracle.kdtree_nn(C, X))
    assert engine.timings()["host_ties"][0] >= 24   # at least every centre row ties


def test_update_exact(engine):
    X, codes = oracle.tile(oracle.gen_image(128), 128, 128, 2, 2)
    engine.set_vectors(X)
    rng = np.random.default_rng(3)
    K = 300
    A = rng.integers(0, K - 20, len(X)).astype(np.uint32)   # some empty cells
    C, cnt = engine.update(A, K)
    np.testing.assert_array_equal(C, oracle.centroids(X, A, K, sum_mode=1))
    np.testing.assert_array_equal(cnt, np.bincount(A, minlength=K))


def test_lbg_zero_rows_and_empty_cells(engine, kdmode):
    """Many all-zero rows (the tiling's end-of-raster padding) and more code vectors than
    distinct rows: empty cells give zero code vectors whose split copies coincide, so
    zero rows tie at several levels.  The result must still match the reference."""
    rng = np.random.default_rng(11)
    X, _ = oracle.tile(oracle.gen_image(64), 64, 64, 2, 2)
    X = X[:300].copy()
    X[rng.choice(300, 120, replace=False)] = 0.0
    C_e, A_k, d_k, _ = reference_lbg(X, 9)
    engine.set_vectors(X)
    C, A, d = engine.lbg(9)
    np.testing.assert_array_equal(A, A_k)
    np.testing.assert_array_equal(C, C_e)
    assert abs(d - d_k) <= 1e-9 * abs(d_k)
    assert sum(engine.timings()["host_ties"]) > 0


@pytest.mark.parametrize("bw,bh", [(1, 1), (2, 3), (3, 3), (4, 2), (4, 4)])
@pytest.mark.parametrize("K", [32, 100, 700])
def test_assign_wide_mfma(engine, monkeypatch, bw, bh, K):
    """The MFMA search for D != 12 (k_wide.hip): codebook resident in LDS or streamed in
    slices (K=700 at D=48 streams, with a partial last slice), K not a multiple of 32
    (padding code vectors), split pairs and duplicates.  Same answer as the reference
    kd-tree and as the VALU search."""
    S = 96
    X, _ = oracle.tile(oracle.gen_image(S), S, S, bw, bh)
    engine.set_vectors(X)
    rng = np.random.default_rng(K + 10 * bw + bh)
    n = (K - 8) // 2
    base = X[rng.choice(len(X), n, replace=True)]
    C = np.concatenate([base * (1 + 0.2), base * (1 - 0.2), np.zeros((4, X.shape[1])), base[:4]])[:K]
    want = oracle.kdtree_nn(C, X)
    np.testing.assert_array_equal(engine.assign(C), want)
    monkeypatch.setenv("QVQ_SEARCH", "valu")
    np.testing.assert_array_equal(engine.assign(C), want)
