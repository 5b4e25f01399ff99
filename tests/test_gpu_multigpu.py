"""The collective path (RCCL) and the C5 configuration on one GPU.

BASELINE.json config 5 / SURVEY.md 8(e): 64 synthetic 4096^2 images (seeds 0x5EED..+63), 2x2
blocks, 1024 code vectors, ONE joint codebook over the image-major concatenation.  On one
MI355X the whole batch (268M blocks, 3.2 GB of codes) fits, so the 8-GPU case's per-level
exchange runs here through a real one-rank RCCL communicator (qvq_comm_init(1, 0)), and the
results must equal the communicator-free run bit for bit -- the property that makes the
1/2/4/8-GPU codebooks identical (exact integer sums).  The reference loops
being sharded are src/Quantizer.cpp:24-32 (assign) and :72-87 (centroids)."""
import json
import os
import subprocess
import time
import sys

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


def _run_ranks(world, case, tmp_path, env=None, limit=150):
    """world rank processes (tests/helpers/rank_worker.py) sharing GPU 0 through the host
    communicator; returns each rank's results.  A rank that fails ends the others at once, and the
    whole group is bounded by `limit` seconds."""
    rdv = str(tmp_path / "rendezvous")
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "helpers", "rank_worker.py")
    outs = [str(tmp_path / ("rank%d.npz" % r)) for r in range(world)]
    penv = dict(os.environ, **(env or {}))
    procs = [subprocess.Popen([sys.executable, worker, str(r), str(world), rdv, case, outs[r]], env=penv)
             for r in range(world)]
    deadline = time.time() + limit
    try:
        while any(p.poll() is None for p in procs):
            if any(p.poll() not in (None, 0) for p in procs) or time.time() > deadline:
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    codes = [p.returncode for p in procs]
    assert codes == [0] * world, codes
    return [dict(np.load(o)) for o in outs]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_ranks_bit_identical_c2(engine, tmp_path, world):
    """The N>1 schedule executed: C2's rows split over `world` processes (contiguous ranges,
    one shared GPU, the per-level exchange through gloo).  Every rank gets the 1-rank codebook
    and distortion bit for bit, the ranks' indices concatenate to the 1-rank indices, and all
    equal the oracle's reference (Kahan) rule."""
    X, _ = oracle.tile(oracle.gen_image(512, 0x5EED), 512, 512, 2, 2)
    engine.set_vectors(X)
    C0, A0, d0 = engine.lbg(10)
    C_x, A_x, d_x = oracle.lbg(X, 10, sum_mode=1)
    _, A_k, _ = oracle.lbg(X, 10, sum_mode=0)
    np.testing.assert_array_equal(A0, A_k)
    np.testing.assert_array_equal(A_k, A_x)
    np.testing.assert_array_equal(C0, C_x)
    res = _run_ranks(world, "c2", tmp_path)
    for r in res:
        assert r["info"][0] == world and r["info"][2] == 2   # host communicator, world ranks
        np.testing.assert_array_equal(r["C"], C0)
        np.testing.assert_array_equal(r["C2"], C0)
        assert float(r["d"][0]) == d0
        assert int(r["cnt"].sum()) == X.shape[0]
    np.testing.assert_array_equal(np.concatenate([r["A"] for r in res]), A0)


@pytest.mark.timeout(300)
def test_sharded_ranks_bit_identical_c5_slice(engine, tmp_path):
    """The reduced C5 batch (4 x 512^2) with whole images per rank, world 2: identical to the
    one-rank run over the concatenation and to the oracle."""
    engine.set_synthetic(512, 0x5EED, 4, 2, 2)
    C0, A0, d0 = engine.lbg(10)
    imgs = [oracle.gen_image(512, 0x5EED + b) for b in range(4)]
    X = np.concatenate([oracle.tile(im, 512, 512, 2, 2)[0] for im in imgs])
    C_x, A_x, _ = oracle.lbg(X, 10, sum_mode=1)
    _, A_k, _ = oracle.lbg(X, 10, sum_mode=0)
    np.testing.assert_array_equal(A0, A_k)   # the reference rule
    np.testing.assert_array_equal(C0, C_x)
    res = _run_ranks(2, "c5", tmp_path)
    for r in res:
        np.testing.assert_array_equal(r["C"], C0)
        assert float(r["d"][0]) == d0
    np.testing.assert_array_equal(np.concatenate([r["A"] for r in res]), A0)


def test_failed_wait_poisons_the_context():
    """a bounded wait that fails while work is still queued must not let results land
    in caller memory later nor let the next call reuse the context's scratch under running kernels.
    A 128-image quantize (~130 ms; the wait consults its deadline every 20 ms) against a 1 us timeout: the call fails, the context refuses
    further work with QVQ_ESTATE, and a fresh context works."""
    import quant_amd
    with quant_amd.Engine(0) as eng:
        eng.set_synthetic(4096, 0x5EED, 128, 2, 2)
        eng.set_timeout(1e-6)
        with pytest.raises(quant_amd.QVQError) as e:
            eng.lbg(10, want_assign=False)
        assert e.value.status == 3   # QVQ_EDEVICE: timed out without a communicator
        with pytest.raises(quant_amd.QVQError) as e2:
            eng.lbg(10, want_assign=False)
        assert e2.value.status == 6   # QVQ_ESTATE
    with quant_amd.Engine(0) as eng:
        eng.set_synthetic(512, 0x5EED, 1, 2, 2)
        C, A, d = eng.lbg(4)
        assert A.max() < 16


CORPUS = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kahan_divergent.json")))
CASES = CORPUS["noise_seeds"] + CORPUS["found"]


def _corpus_expect(engine):
    """Per corpus case: the tiled rows, the oracle's reference (Kahan) rule, and the one-rank
    engine's results."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "helpers"))
    from kahan_env_worker import make
    out = []
    for c in CASES:
        X, _ = oracle.tile(make(c), c["side"], c["side"], c["bw"], c["bh"])
        _, A_k, _ = oracle.lbg(X, c["bits"], sum_mode=0)
        _, A_x, _ = oracle.lbg(X, c["bits"], sum_mode=1)
        engine.set_vectors(X)
        C0, A0, d0 = engine.lbg(c["bits"])
        np.testing.assert_array_equal(A0, A_k)
        out.append((X, A_k, A_x, C0, d0))
    return out


@pytest.fixture(scope="module")
def corpus_expect(engine):
    return _corpus_expect(engine)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_ranks_follow_the_kahan_rule_on_the_corpus(corpus_expect, tmp_path, world):
    """with a communicator the indices follow the reference's rule.  Every
    case of the divergent corpus (the exact-sum rule's indices differ from the reference's there)
    with its rows split over `world` processes: the ranks' indices concatenate to the oracle's
    Kahan-rule indices, every rank's codebook and distortion equal the one-rank run's bit for
    bit, and qvq_update_kahan of the local indices returns the reference's centroids over all the
    rows (cells' chains across ranks, src/Quantizer.cpp:59-70)."""
    res = _run_ranks(world, "corpus", tmp_path)
    relays = 0
    for i, (X, A_k, A_x, C0, d0) in enumerate(corpus_expect):
        assert not np.array_equal(A_k, A_x)
        bits = CASES[i]["bits"]
        np.testing.assert_array_equal(np.concatenate([r["A%d" % i] for r in res]), A_k, err_msg="case %d" % i)
        K_ref = oracle.centroids(X, A_k, 1 << bits, sum_mode=0)
        for r in res:
            np.testing.assert_array_equal(r["C%d" % i], C0, err_msg="case %d" % i)
            assert float(r["d%d" % i][0]) == d0
            np.testing.assert_array_equal(r["K%d" % i].view(np.uint64), K_ref.view(np.uint64), err_msg="case %d" % i)
        relays += int(res[0]["relays%d" % i][0])
        assert len({int(r["redo%d" % i][0]) for r in res}) == 1   # every rank redoes, or none
    assert relays > 0   # some levels needed cells summed across the ranks


@pytest.mark.timeout(300)
def test_one_rank_failure_redoes_every_rank(corpus_expect, tmp_path):
    """A check failing on rank 0 only (QVQ_KAHAN_FAIL_LEVEL / _RANK) makes both ranks redo the
    quantize with synchronous several-rank Kahan levels (the whole reference split summed across
    the ranks on each tie level): same indices, kahan_redo 1 on both."""
    res = _run_ranks(2, "corpus", tmp_path, env={"QVQ_KAHAN_FAIL_LEVEL": "4", "QVQ_KAHAN_FAIL_RANK": "0"})
    redone = 0
    for i, (X, A_k, A_x, C0, d0) in enumerate(corpus_expect):
        np.testing.assert_array_equal(np.concatenate([r["A%d" % i] for r in res]), A_k, err_msg="case %d" % i)
        for r in res:
            np.testing.assert_array_equal(r["C%d" % i], C0, err_msg="case %d" % i)
        rd = {int(r["redo%d" % i][0]) for r in res}
        assert len(rd) == 1
        redone += rd.pop()
    assert redone >= len([c for c in CASES if c["bits"] >= 4])


@pytest.mark.timeout(300)
def test_open_row_without_cells_redoes_every_rank(corpus_expect, tmp_path):
    """a deferred check whose open rows want no cell (nothing summed over the ranks can
    settle them) must fail the level, not be skipped at the vote with its speculative indices kept.
    QVQ_KAHAN_OPEN_LEVEL=-1 leaves a row of every tie level open with no cell wanted, on both
    ranks: every corpus case (each has tie rows) redoes the quantize and still returns the
    reference's indices."""
    res = _run_ranks(2, "corpus", tmp_path, env={"QVQ_KAHAN_OPEN_LEVEL": "-1"})
    redone = 0
    for i, (X, A_k, A_x, C0, d0) in enumerate(corpus_expect):
        np.testing.assert_array_equal(np.concatenate([r["A%d" % i] for r in res]), A_k, err_msg="case %d" % i)
        for r in res:
            np.testing.assert_array_equal(r["C%d" % i], C0, err_msg="case %d" % i)
        rd = {int(r["redo%d" % i][0]) for r in res}
        assert len(rd) == 1
        redone += rd.pop()
    assert redone == len(CASES)
