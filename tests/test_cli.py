"""The command-line front end (quant_amd/lib/quant): the reference's flags, defaults and
file-type dispatch (src/main.cpp:42-113) over libquant_amd.so.

CPU: help text, argument errors and the "File type not supported" path (no GPU needed).
GPU: ppm -> quant, quant -> ppm and ppm -> ppm (with the raport) byte-for-byte against the
oracle's restatement of compress / saveToFile / decompress."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, load_png_rgb
from oracle import oracle

QUANT = os.path.join(ROOT, "quant_amd", "lib", "quant")


def run(*args, timeout=300):
    if not os.path.exists(QUANT):
        pytest.fail("quant CLI not built (run __graft_entry__.build())")
    return subprocess.run([QUANT, *map(str, args)], capture_output=True, text=True, timeout=timeout)


def _write_ppm(path, rgb, xs, ys):
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (xs, ys))
        f.write(np.asarray(rgb, np.uint8).tobytes())


def test_help_and_argument_errors(tmp_path):
    r = run("--help")
    assert r.returncode == 0 and "-n arg (=8)" in r.stdout and "Save to" in r.stdout
    assert run("in.ppm").returncode == 2                       # --saveto is required
    assert run("-o", "x.quant").returncode == 2                # the file is required
    assert run("in.ppm", "-o", "x.quant", "-z", "1").returncode == 2
    assert run("in.ppm", "-o", "x.quant", "-r", "maybe").returncode == 2


@pytest.mark.parametrize("src,dst", [("a.png", "b.quant"), ("a.ppm", "b.png"), ("a.quant", "b.quant"),
                                     ("dir.ppm/a", "b.quant")])
def test_unsupported_file_types(tmp_path, src, dst):
    r = run(src, "-o", dst)
    assert r.returncode == 1 and "File type not supported" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name,flags,bits,bw,bh,cs", [
    ("beans.png", [], 8, 2, 2, oracle.SCALED),                              # all defaults
    ("t.png", ["-n6", "-w", "2", "-h3"], 6, 2, 3, oracle.SCALED),           # wrap/pad, short forms
    ("kodim01.png", ["-n", "10", "--colorspace=0", "-e", "0.5"], 10, 2, 2, oracle.NORMAL),
])
def test_cli_round_trips_match_oracle(tmp_path, name, flags, bits, bw, bh, cs):
    rgb, xs, ys = load_png_rgb(name)
    ppm, quant = tmp_path / "in.ppm", tmp_path / "out.quant"
    dec, dec2 = tmp_path / "dec.ppm", tmp_path / "dec2.ppm"
    _write_ppm(ppm, rgb, xs, ys)
    r = run(ppm, "-o", quant, *flags)
    assert r.returncode == 0, r.stderr
    X, _ = oracle.tile(rgb, xs, ys, bw, bh, cs=cs, pad_code=128 if cs == oracle.SCALED else 0)
    C_k, A_k, _ = oracle.lbg(X, bits, sum_mode=0)
    cb = oracle.codebook_bytes(C_k, cs=cs)
    assert open(quant, "rb").read() == oracle.quant_file_bytes(cb, A_k, bits, cs, xs, ys, bw, bh)
    want = oracle.decode(cb, A_k, xs, ys, bw, bh)
    r = run(quant, "-o", dec)                                   # quant -> ppm
    assert r.returncode == 0, r.stderr
    img, dx, dy = oracle.read_ppm(dec)
    assert (dx, dy) == (xs, ys)
    np.testing.assert_array_equal(img, want)
    r = run("--saveto=" + str(dec2), ppm, "-r", "1", *flags)     # ppm -> ppm with the raport
    assert r.returncode == 0, r.stderr
    np.testing.assert_array_equal(oracle.read_ppm(dec2)[0], want)
    lines = dict(ln.split(" = ") for ln in r.stdout.splitlines() if " = " in ln)
    assert abs(float(lines["Distortion       "]) - oracle.raport_distortion(rgb, want)) <= 1e-9
    assert "Compression time " in lines and lines["Compression time "].endswith("s")
