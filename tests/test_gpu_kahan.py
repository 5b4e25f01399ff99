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
    # the closed-form distortion is exact to ~1e-16 of the mean square value (cancellation)
    assert abs(d - d_k) <= 1e-9 * abs(d_k) + 1e-14 * float(np.mean(X * X))
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


# ---- the Kahan centroid evaluator itself (qvq_update_kahan, k_kahan.hip) -------------------------
def _spatial_assign(n, K, seed, run=5000):
    """Cells in runs along the row order (as a real assignment: image regions), some cells empty."""
    rng = np.random.default_rng(seed)
    runs = rng.integers(0, max(1, K - K // 8), (n + run - 1) // run)
    A = np.repeat(runs, run)[:n].astype(np.uint32)
    flip = rng.random(n) < 0.2
    A[flip] = rng.integers(0, K, int(flip.sum()))
    return A


KAHAN_CASES = [
    # (image, side, bw, bh, K, assignment)
    ("noise", 96, 2, 2, 37, "random"),
    ("noise", 96, 1, 1, 1, "mean"),
    ("synthetic", 512, 2, 2, 32, "lbg5"),
    ("synthetic", 512, 2, 2, 512, "lbg9"),
    ("dark", 256, 2, 2, 8, "spatial"),     # values near 0 (tiny grids) and 1.0 (decisions)
    ("synthetic", 4096, 2, 2, 32, "spatial"),
    ("synthetic", 4096, 2, 2, 512, "spatial"),
    ("synthetic", 4096, 2, 2, 1, "mean"),
    ("synthetic", 1024, 4, 4, 64, "spatial"),
]


def _kahan_input(case):
    img, side, bw, bh, K, how = case
    if img == "noise":
        rgb = np.random.default_rng(7).integers(0, 256, side * side * 3, dtype=np.uint8)
    elif img == "dark":
        rng = np.random.default_rng(3)
        # raw bytes 127 (value 1.0), 128..131 (values 0..3/255) and a few others, in regions
        base = np.where((np.arange(side * side * 3) // 5000) % 2, 127, 128).astype(np.int64)
        rgb = (base + rng.integers(0, 4, side * side * 3) * (base == 128)).astype(np.uint8)
        mask = rng.random(rgb.size) < 0.01
        rgb[mask] = rng.integers(0, 256, int(mask.sum()))
    else:
        rgb = oracle.gen_image(side)
    X, _ = oracle.tile(rgb, side, side, bw, bh)
    n = X.shape[0]
    if how == "random":
        A = np.random.default_rng(1).integers(0, K - 3, n).astype(np.uint32)   # the last cells empty
    elif how == "mean":
        A = np.zeros(n, np.uint32)
    elif how.startswith("lbg"):
        _, _, _, _, assigns = oracle.lbg(X, int(how[3:]), sum_mode=0, threads=8, dump=True)
        A = assigns[-1].astype(np.uint32)
    else:
        A = _spatial_assign(n, K, seed=side + K)
    return rgb, X, A


@pytest.mark.parametrize("case", KAHAN_CASES, ids=lambda c: "-".join(str(x) for x in c))
def test_kahan_centroids_are_the_reference_bits(engine, case):
    img, side, bw, bh, K, how = case
    rgb, X, A = _kahan_input(case)
    engine.set_images(rgb, 1, side, side, bw, bh, oracle.SCALED)
    C = engine.update_kahan(A, K)
    C_ref = oracle.centroids(X, A, K, sum_mode=0)
    np.testing.assert_array_equal(C.view(np.uint64), C_ref.view(np.uint64))


def _cuts(n, rng, pieces):
    """Row offsets cutting n rows into `pieces` ranks: some cuts early (inside the chains' double
    transient), some repeated (a rank without rows), some at the end."""
    c = [0, n]
    for p in range(pieces - 1):
        r = rng.random()
        c.append(int(rng.integers(0, min(n, 40) + 1)) if r < 0.3 else n if r < 0.4 else int(rng.integers(0, n + 1)))
    return np.array(sorted(c), np.uint64)


@pytest.mark.parametrize("case", KAHAN_CASES, ids=lambda c: "-".join(str(x) for x in c))
def test_chained_kahan_centroids_are_the_reference_bits(engine, case):
    """a cell's Kahan chain split over ranks (k_kahan.hip chained evaluation: each
    rank's functions built at the chain's global prefix, the state (sum, c) handed from rank to
    rank), here as virtual ranks on one device at random cuts -- the reference's bits for every
    cut (src/Quantizer.cpp:59-70 sums the cell's rows in ascending order over all of them)."""
    img, side, bw, bh, K, how = case
    rgb, X, A = _kahan_input(case)
    engine.set_images(rgb, 1, side, side, bw, bh, oracle.SCALED)
    C_ref = oracle.centroids(X, A, K, sum_mode=0).view(np.uint64)
    rng = np.random.default_rng(side * 131 + K)
    n = X.shape[0]
    for pieces in (2, 3, 5, 8):
        cuts = _cuts(n, rng, pieces)
        C = engine.update_kahan_split(A, K, cuts)
        np.testing.assert_array_equal(C.view(np.uint64), C_ref, err_msg="cuts %s" % cuts.tolist())


CORPUS_SUBSET = CORPUS["noise_seeds"] + CORPUS["found"][::4]


@pytest.mark.parametrize("case", CORPUS_SUBSET, ids=lambda c: "%s-%d-%d-%dx%d-n%d" % (
    c["kind"], c["seed"], c["side"], c["bw"], c["bh"], c["bits"]))
def test_corpus_through_one_rank_communicator(engine, case):
    """The verdict's r04 gap: with a communicator the indices must follow the reference's rule
    too.  A one-rank RCCL communicator runs the collective schedule; its codebook and indices
    equal the communicator-free run's (and the oracle's Kahan rule)."""
    import quant_amd
    rgb = _make(case)
    side, bw, bh, bits = case["side"], case["bw"], case["bh"], case["bits"]
    engine.set_images(rgb, 1, side, side, bw, bh, oracle.SCALED)
    C0, A0, d0 = engine.lbg(bits)
    with quant_amd.Engine(0) as eng:
        eng.comm_init(1, 0, quant_amd.Engine.comm_unique_id())
        assert _check(eng, case) > 0
        C1, A1, d1 = eng.lbg(bits)
    np.testing.assert_array_equal(A1, A0)
    np.testing.assert_array_equal(C1, C0)
    assert d1 == d0


def _env_worker(env, cases):
    import subprocess
    import sys
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "helpers", "kahan_env_worker.py")
    r = subprocess.run([sys.executable, worker, json.dumps(cases)], env=dict(os.environ, **env), capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]


def test_synchronous_kahan_levels_follow_the_reference_rule():
    """the synchronous Kahan path (QVQ_SPECULATE=0: every tie level's ties answered
    by the certificate or the whole reference-bit split before the level finishes) on corpus
    cases, in a process of its own (the switch is read once)."""
    res = _env_worker({"QVQ_SPECULATE": "0"}, CORPUS["noise_seeds"][:2] + CORPUS["found"][:6])
    assert len(res) == 8
    for r in res:
        assert r["A_ok"] and r["C_ok"] and r["again_ok"], r
        assert r["redo"] == 0


def test_failed_check_redoes_the_quantize():
    """a speculative check that fails (forced at level 6, QVQ_KAHAN_FAIL_LEVEL) makes
    the quantize run again with synchronous Kahan levels: kahan_redo == 1, the indices are still
    the reference's, and a second quantize on the same context agrees."""
    res = _env_worker({"QVQ_KAHAN_FAIL_LEVEL": "6"}, CORPUS["noise_seeds"][:1] + [
        dict(kind="gen", seed=0x5EED, side=256, bw=2, bh=2, bits=8)])
    for r in res:
        assert r["A_ok"] and r["C_ok"] and r["again_ok"], r
        assert r["redo"] == 1


def test_certificate_cells_through_segment_functions():
    """The certificate's cell sums with the step-by-step chains off (QVQ_KAHAN_DIRECT_MAX=0:
    every chain through the segment functions, as for long cells), on corpus cases whose
    checks sum cells: the same indices and codebooks (the default run takes ks_direct_kernel
    for their short cells)."""
    res = _env_worker({"QVQ_KAHAN_DIRECT_MAX": "0"}, CORPUS["noise_seeds"][:2] + CORPUS["found"][:6])
    assert len(res) == 8
    for r in res:
        assert r["A_ok"] and r["C_ok"] and r["again_ok"], r


def test_late_tree_job_reads_its_own_codebook():
    """the r05m race made deterministic.  A synchronous level's tree job
    copies the codebook its level's search ran on from mapped memory, while the main thread has
    already enqueued the level's own finalize, which publishes the next level's codebook.
    QVQ_TREE_JOB_DELAY_MS=20 makes every job late past that finalize.  With the published codebooks
    double-buffered by level parity (the fix, fc64269) the indices are the reference's; with the one
    buffer of before (QVQ_CB_SINGLE=1, test only) the late jobs build their trees over the next
    level's code vectors and some tie rows come out wrong."""
    cases = CORPUS["noise_seeds"][:2] + CORPUS["found"][:6]
    good = _env_worker({"QVQ_SPECULATE": "0", "QVQ_TREE_JOB_DELAY_MS": "20"}, cases)
    assert len(good) == len(cases)
    for r in good:
        assert r["A_ok"] and r["C_ok"] and r["again_ok"], r
    bad = _env_worker({"QVQ_SPECULATE": "0", "QVQ_TREE_JOB_DELAY_MS": "20", "QVQ_CB_SINGLE": "1"}, cases)
    assert len(bad) == len(cases)
    assert any(not (r["A_ok"] and r["again_ok"]) for r in bad), "the single buffer should show the race"
