"""The pruned MFMA search (k_mf32.hip PRUNE, K >= 512 at D = 12): a chunk of 64 rows visits its
code tiles outward from its projection on the all-ones direction and stops once the tiles left are
provably farther than every row's current best (||x - c||^2 >= (sum_d (x_d - c_d))^2 / D).  The
skipped code vectors can be no row's answer nor tie with it, so indices and codebook must equal the
reference rule on data that stresses the bound: pure noise (wide bounds, little pruning), smooth
gradients (tight bounds, heavy pruning), flat regions with many duplicate rows and exact ties,
and NORMAL values.  Reference: src/Quantizer.cpp:24-32 (assign), nanoflann.hpp:320-345."""
import numpy as np
import pytest

from conftest import reference_lbg
from oracle import oracle

pytestmark = pytest.mark.gpu


def _image(kind, S, seed=1):
    rng = np.random.default_rng(seed)
    if kind == "noise":
        return rng.integers(0, 256, size=S * S * 3, dtype=np.uint8)
    r, c = np.meshgrid(np.arange(S), np.arange(S), indexing="ij")
    if kind == "smooth":
        img = np.stack([r * 255 // (S - 1), c * 255 // (S - 1), (r + c) * 255 // (2 * S - 2)], -1)
        return img.astype(np.uint8).ravel()
    if kind == "flat":   # 16 x 16 constant patches of 8 colours plus a few noisy rows
        pal = rng.integers(0, 256, size=(8, 3))
        img = pal[((r // 16) * 3 + (c // 16)) % 8].astype(np.uint8)
        img[::37] = rng.integers(0, 256, size=img[::37].shape, dtype=np.uint8)
        return img.ravel()
    raise ValueError(kind)


@pytest.mark.parametrize("kind,cs", [("noise", oracle.SCALED), ("smooth", oracle.SCALED), ("flat", oracle.SCALED),
                                     ("smooth", oracle.NORMAL)])
def test_pruned_search_matches_reference(engine, kind, cs):
    import quant_amd
    S = 256
    rgb = _image(kind, S)
    X, _ = oracle.tile(rgb, S, S, 2, 2, cs=cs, pad_code=128 if cs == oracle.SCALED else 0)
    C_e, A_k, d_k, _ = reference_lbg(X, 10)
    engine.set_images(rgb, 1, S, S, 2, 2, quant_amd.SCALED if cs == oracle.SCALED else quant_amd.NORMAL)
    C, A, d = engine.lbg(10)
    np.testing.assert_array_equal(A, A_k)
    np.testing.assert_array_equal(C, C_e)
    assert abs(d - d_k) <= 1e-9 * abs(d_k)


# The wide search (D = 48, 4x4 blocks) prunes from K = 1024 with streamed codebook slices: a
# workgroup's 8 chunks stacked down the image columns share one window of slices (k_wide.hip
# PRUNE).  Same reference rule; the set_vectors case has no image geometry (consecutive chunks).
@pytest.mark.parametrize("kind,S,bits,vectors", [("smooth", 512, 12, False), ("flat", 512, 12, False),
                                                 ("noise", 512, 11, False), ("smooth", 1024, 11, True)])
def test_wide_pruned_search_matches_reference(engine, kind, S, bits, vectors):
    import quant_amd
    rgb = _image(kind, S, seed=3)
    X, _ = oracle.tile(rgb, S, S, 4, 4)
    C_e, A_k, d_k, _ = reference_lbg(X, bits)
    if vectors:
        engine.set_vectors(X)
    else:
        engine.set_images(rgb, 1, S, S, 4, 4, quant_amd.SCALED)
    C, A, d = engine.lbg(bits)
    np.testing.assert_array_equal(A, A_k)   # the reference rule (this case's exact-sum rule differs)
    np.testing.assert_array_equal(C, C_e)
    assert abs(d - d_k) <= 1e-9 * abs(d_k)
