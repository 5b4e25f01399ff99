"""Host C++ under AddressSanitizer + UndefinedBehaviorSanitizer (VERDICT r02
missing #3).  tests/cpp/Makefile builds the product's host code -- the reference kd-tree
(quant_amd/csrc/kdtree.cpp), the bounded-wait policy (wait.hpp), the codec (quant_amd/cpp/*.cpp:
.quant writer/reader, PPM IO, colour spaces, tiling) and the CLI (quant_amd/cli/quant.cpp) -- with
-fsanitize=address,undefined (UB fatal, leak checking on).  The driver checks the kd-tree against
the oracle, the wait policy under scripted probes and the codec round trips; the CLI runs its
argument, file and error paths.  CPU only: the engine calls are linked but fail cleanly without a
GPU (qvq_create), which is itself one of the exercised paths."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "cpp", "build-san")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


@pytest.fixture(scope="module")
def san_build():
    if not os.path.exists(os.path.join(ROOT, "quant_amd", "lib", "libqvq.so")):
        pytest.skip("libqvq.so not built")
    r = subprocess.run(["make", "-s", "-j4", "-C", os.path.join(ROOT, "tests", "cpp")], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return BUILD


def _clean(out):
    assert "ERROR: AddressSanitizer" not in out and "ERROR: LeakSanitizer" not in out, out[-3000:]
    assert "runtime error:" not in out, out[-3000:]


def test_host_code_under_sanitizers(san_build, tmp_path):
    r = subprocess.run([os.path.join(san_build, "test_host_sanitize"), str(tmp_path)], capture_output=True, text=True,
                       timeout=600, env=ENV)
    _clean(r.stdout + r.stderr)
    assert r.returncode == 0 and "host sanitize test: ok" in r.stdout, r.stdout + r.stderr


def test_cli_paths_under_sanitizers(san_build, tmp_path):
    q = os.path.join(san_build, "quant")
    ppm = tmp_path / "t.ppm"
    ppm.write_bytes(b"P6\n4 3\n255\n" + bytes(range(36)))
    bad = tmp_path / "bad.quant"
    bad.write_bytes(b"4 1 6 4 3 2 2\n" + bytes(10))   # truncated codebook
    cases = [  # (argv, expected exit status)
        (["--help"], 0),
        ([], 2),                                   # --file missing
        (["-n"], 2),                               # value missing
        (["-nX", str(ppm), "-o", "o.quant"], 2),   # not an integer
        (["-r", "maybe", str(ppm), "-o", "o.quant"], 2),
        ([str(ppm), str(ppm), "-o", "o.quant"], 2),   # two files
        (["a.txt", "-o", "b.txt"], 1),             # file types
        ([str(tmp_path / "missing.ppm"), "-o", "o.quant"], 3),
        ([str(bad), "-o", str(tmp_path / "o.ppm")], 3),   # truncated .quant
        ([str(ppm), "-o", str(tmp_path / "o.quant"), "-r", "1"], (0, 3)),   # compress: 3 without a GPU
    ]
    for argv, want in cases:
        r = subprocess.run([q] + argv, capture_output=True, text=True, timeout=120, env=ENV, cwd=tmp_path)
        _clean(r.stdout + r.stderr)
        assert r.returncode in (want if isinstance(want, tuple) else (want,)), (argv, r.returncode, r.stderr[-2000:])
