"""CPU checks of the Kahan-bit machinery (no GPU).

* quant_amd/csrc/kahan_par.hpp: the device pipeline restated serially on the CPU (segment
  metadata, prefix sums, segment functions, 64-segment block composites, the checked evaluation
  with replays, tests/cpp/test_kahan_chain.cpp) returns the bits of the reference's sequential
  Kahan chain (sumInArea, src/Quantizer.cpp:59-70) on random chains of ten kinds and on the
  chains of a real assignment (the oracle's level-5 cells of the synthetic image).
* quant_amd/csrc/kdtree.cpp RefKDTree::unchanged_under: never claims that the Kahan-bit split's
  tree equals the exact-sum split's when the images differ (tests/cpp/test_kdtree_reuse.cpp)."""
import os
import struct
import subprocess

import numpy as np
import pytest

from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "quant_amd", "csrc")
CPP = os.path.join(ROOT, "tests", "cpp")


def _build(tmp_path, name, extra=()):
    exe = str(tmp_path / name)
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-I", CSRC, "-o", exe, os.path.join(CPP, name + ".cpp"), *extra],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


@pytest.fixture(scope="module")
def s512():
    rgb = oracle.gen_image(512)
    X, codes = oracle.tile(rgb, 512, 512, 2, 2)
    C0, A0, d0, sp0, as0 = oracle.lbg(X, 9, sum_mode=0, threads=8, dump=True)
    _, _, _, sp1, _ = oracle.lbg(X, 9, sum_mode=1, threads=8, dump=True)
    return codes, as0, sp0, sp1


def test_kahan_chain_random(tmp_path):
    exe = _build(tmp_path, "test_kahan_chain")
    r = subprocess.run([exe, "150"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr


def test_kahan_chain_real_assignment(tmp_path, s512):
    codes, as0, _, _ = s512
    A = as0[4]   # level 5: 32 cells
    order = np.argsort(A, kind="stable")
    koff = np.searchsorted(A[order], np.arange(33))
    path = tmp_path / "chains.bin"
    with open(path, "wb") as f:
        f.write(struct.pack("<I", 32 * 12))
        for k in range(32):
            rows = order[koff[k]:koff[k + 1]]
            for d in range(12):
                c = codes[rows, d].astype(np.uint8)
                f.write(struct.pack("<I", len(c)))
                f.write(c.tobytes())
    exe = _build(tmp_path, "test_kahan_chain")
    r = subprocess.run([exe, str(path)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr


def test_kdtree_reuse_is_sound(tmp_path, s512):
    _, _, sp0, sp1 = s512
    path = tmp_path / "pairs.bin"
    with open(path, "wb") as f:
        for kahan, exact in zip(sp0, sp1):
            f.write(struct.pack("<II", kahan.shape[0], kahan.shape[1]))
            f.write(np.ascontiguousarray(exact, np.float64).tobytes())
            f.write(np.ascontiguousarray(kahan, np.float64).tobytes())
    exe = _build(tmp_path, "test_kdtree_reuse", [os.path.join(CSRC, "kdtree.cpp")])
    r = subprocess.run([exe, str(path)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "wrong claims 0" in r.stdout, r.stdout + r.stderr


def test_tie_certificate_is_sound(tmp_path):
    """quant_amd/csrc/kdtree.cpp certified_search: answering tie rows from the
    exact-sum split's tree, with the reference's bits computed only for the candidates' cells,
    never gives an index other than the reference's (the synthetic image's levels with extra
    ordinary rows, and the four noise seeds of the Kahan corpus)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import json
    from tie_cert_data import write_levels
    rng = np.random.default_rng(5)
    path = tmp_path / "levels.bin"
    with open(path, "wb") as f:
        X, _ = oracle.tile(oracle.gen_image(512), 512, 512, 2, 2)
        write_levels(f, X, 9, 100, rng)
        corpus = json.load(open(os.path.join(ROOT, "tests", "golden", "kahan_divergent.json")))
        for case in corpus["noise_seeds"]:
            rgb = np.random.default_rng(case["seed"]).integers(0, 256, 96 * 96 * 3, dtype=np.uint8)
            X, _ = oracle.tile(rgb, 96, 96, 2, 2)
            write_levels(f, X, case["bits"], 20, rng)
    exe = _build(tmp_path, "test_tie_cert", [os.path.join(CSRC, "kdtree.cpp")])
    r = subprocess.run([exe, str(path)], capture_output=True, text=True, timeout=600)
    last = r.stdout.strip().splitlines()[-1]
    assert r.returncode == 0 and " wrong 0 " in last and "delta 0" in last, r.stdout[-3000:] + r.stderr
    certified = int(last.split("certified ")[1].split()[0])
    assert certified > 0, last
