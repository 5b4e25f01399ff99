"""The collective path (RCCL) and the C5 configuration on one GPU.

BASELINE.json config 5 / SURVEY.md 8(e): 64 synthetic 4096^2 images (seeds 0x5EED..+63), 2x2
blocks, 1024 code vectors, ONE joint codebook over the image-major concatenation.  On one
MI355X the whole batch (268M blocks, 3.2 GB of codes) fits, so the 8-GPU case's per-level
exchange runs here through a real one-rank RCCL communicator (qvq_comm_init(1, 0)), and the
results must equal the communicator-free run bit for bit -- the property that makes the
1/2/4/8-GPU codebooks identical (exact integer sums).  The reference loops
being sharded are src/Quantizer.cpp:24-32 (assign) and :72-87 (centroids)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _comm_engine(dev=0):
    import quant_amd
    eng = quant_amd.Engine(dev)
    eng.comm_init(1, 0, quant_amd.Engine.comm_unique_id())
    return eng


def test_one_rank_communicator_is_bit_identical(engine):
    engine.set_synthetic(512, 0x5EED, 2, 2, 2)
    C0, A0, d0 = engine.lbg(10)
    with _comm_engine() as eng:
        eng.set_synthetic(512, 0x5EED, 2, 2, 2)
        C1, A1, d1 = eng.lbg(10)
        np.testing.assert_array_equal(A0, A1)
        np.testing.assert_array_equal(C0, C1)
        assert d0 == d1
        # the single-step update also goes through the all-reduce
        C2, cnt = eng.update(A1, 1 << 10)
        np.testing.assert_array_equal(C2, C1)


def test_c5_reduced_batch_matches_oracle():
    """C5 parity on a reduced batch -- 4 x 512^2 images concatenated,
    through the communicator path, against the oracle's LBG over the same rows."""
    imgs = [oracle.gen_image(512, 0x5EED + b) for b in range(4)]
    X = np.concatenate([oracle.tile(im, 512, 512, 2, 2)[0] for im in imgs])
    C_x, A_x, d_x = oracle.lbg(X, 10, sum_mode=1)
    C_k, A_k, _ = oracle.lbg(X, 10, sum_mode=0)
    with _comm_engine() as eng:
        eng.set_synthetic(512, 0x5EED, 4, 2, 2)
        C, A, d = eng.lbg(10)
    np.testing.assert_array_equal(A, A_k)        # the reference rule (Kahan sums) ...
    np.testing.assert_array_equal(A, A_x)        # ... and the exact-sum rule agree here
    np.testing.assert_array_equal(C, C_x)
    assert abs(d - d_x) <= 1e-9 * abs(d_x)


def test_c5_full_batch_properties():
    """Full C5 (64 x 4096^2, 2x2, K=1024) on one GPU, through the communicator: the Lloyd
    fixed point (the returned codebook is exactly the centroid map of the returned
    assignment), determinism, and equality with the communicator-free run."""
    import quant_amd
    S, n_img, bits = 4096, 64, 10
    with _comm_engine() as eng:
        eng.set_synthetic(S, 0x5EED, n_img, 2, 2)
        assert eng.n == n_img * (S // 2) ** 2
        C, A, d = eng.lbg(bits)
        assert A.max() < (1 << bits)
        C2, cnt = eng.update(A, 1 << bits)
        np.testing.assert_array_equal(C, C2)
        assert int(cnt.sum()) == eng.n
        C3, A3, d3 = eng.lbg(bits, want_assign=False)
        np.testing.assert_array_equal(C, C3)
        assert d3 == d
        h_first = oracle.sha16(A)
    with quant_amd.Engine(0) as eng:
        eng.set_synthetic(S, 0x5EED, n_img, 2, 2)
        C4, A4, d4 = eng.lbg(bits)
        np.testing.assert_array_equal(C, C4)
        assert oracle.sha16(A4) == h_first
