"""The C++ API (include/quant_amd/*.hpp over libqvq.so): the reference's Quantizer /
CompressedImage interface, driven through tests/cpp/test_api.cpp.

CPU: the reference's own tiling round-trip cases (src/test.cpp), .quant / PPM round trips,
colour maps, report text.  GPU: CompressedImage::compress and getQuantizer(LBG)->quantize
against the oracle -- .quant bytes, decoded image and report distortion."""
import os
import subprocess

import numpy as np
import pytest

from conftest import load_png_rgb
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "quant_amd", "lib")


@pytest.fixture(scope="module")
def test_api(tmp_path_factory):
    if not os.path.exists(os.path.join(LIB, "libquant_amd.so")):
        pytest.fail("libquant_amd.so not built (run __graft_entry__.build())")
    exe = str(tmp_path_factory.mktemp("cpp") / "test_api")
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "test_api.cpp"), "-L" + LIB, "-lquant_amd", "-lqvq",
                    "-Wl,-rpath," + LIB, "-o", exe], check=True)
    return exe


def test_host_api(test_api, tmp_path):
    r = subprocess.run([test_api, "host", str(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_exports_cpp_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(LIB, "libquant_amd.so")],
                         capture_output=True, text=True, check=True).stdout
    for sym in ["getQuantizer", "getColorSpace", "CompressedImage8compress", "CompressedImage10decompress",
                "CompressedImage10saveToFile", "CompressedImage12loadFromFile", "getBlocksAsVectorsFromImage",
                "vectorsToCharVectorsColorSpaced", "getImageFromVectors"]:
        assert sym in out, sym


def _write_ppm(path, rgb, xs, ys):
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (xs, ys))
        f.write(np.asarray(rgb, np.uint8).tobytes())


@pytest.mark.gpu
@pytest.mark.parametrize("name,bits,bw,bh", [("beans.png", 8, 2, 2), ("kodim01.png", 10, 2, 2),
                                             ("t.png", 6, 2, 3)])
def test_compress_matches_oracle(test_api, tmp_path, name, bits, bw, bh):
    rgb, xs, ys = load_png_rgb(name)
    ppm, quant, dec = str(tmp_path / "in.ppm"), str(tmp_path / "out.quant"), str(tmp_path / "dec.ppm")
    _write_ppm(ppm, rgb, xs, ys)
    r = subprocess.run([test_api, "compress", ppm, quant, dec, str(bits), str(bw), str(bh), "1"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    X, _ = oracle.tile(rgb, xs, ys, bw, bh)
    C_k, A_k, _ = oracle.lbg(X, bits, sum_mode=0)
    C_x, A_x, _ = oracle.lbg(X, bits, sum_mode=1)
    np.testing.assert_array_equal(A_k, A_x)
    cb = oracle.codebook_bytes(C_x)
    np.testing.assert_array_equal(cb, oracle.codebook_bytes(C_k))   # reference's centroids: same bytes
    expected = oracle.quant_file_bytes(cb, A_k, bits, 1, xs, ys, bw, bh)
    got = open(quant, "rb").read()
    assert got == expected
    dec_rgb, dx, dy = oracle.read_ppm(dec)
    assert (dx, dy) == (xs, ys)
    want = oracle.decode(cb, A_k, xs, ys, bw, bh)
    np.testing.assert_array_equal(dec_rgb, want)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("Distortion")][0]
    assert abs(float(line.split("=")[1]) - oracle.raport_distortion(rgb, want)) <= 1e-9


@pytest.mark.gpu
def test_quantizer_plugin_matches_oracle(test_api, tmp_path):
    X, _ = oracle.tile(oracle.gen_image(96), 96, 96, 2, 2, cs=oracle.NORMAL, pad_code=0)
    xf, cf, af = tmp_path / "x.f64", tmp_path / "c.f64", tmp_path / "a.u32"
    X.astype(np.float64).tofile(xf)
    r = subprocess.run([test_api, "quantize", str(xf), str(X.shape[0]), str(X.shape[1]), "7", str(cf), str(af)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    C_x, A_x, d_x = oracle.lbg(X, 7, sum_mode=1)
    np.testing.assert_array_equal(np.fromfile(af, np.uint32), A_x)
    np.testing.assert_array_equal(np.fromfile(cf, np.float64).reshape(C_x.shape), C_x)
    assert abs(float(r.stdout.split()[1]) - d_x) <= 1e-9 * abs(d_x)


@pytest.mark.gpu
def test_compress_near_byte_flip_takes_reference_bits(test_api, tmp_path):
    """the .quant codebook bytes are round((c - 128) * 255) of the reference's
    Kahan centroids (src/ColorSpace.cpp:23-28, src/Compressor.cpp:12-29).  The engine's exact-sum
    centroids can differ by a few ulps, so compress fetches the reference's bits (qvq_update_kahan)
    whenever a component lies within 16 ulps of a point where the byte changes.  Here one cell's
    mean is exactly 117.5 / 255 in every channel (rows at u = 117 and 118, half each), the
    neighbourhood of such a point: the file must hold the Kahan oracle's bytes."""
    S = 64
    rng = np.random.default_rng(117)
    n = S * S
    u = np.empty((n, 3), np.int64)
    dark = np.zeros(n, bool)
    dark[rng.permutation(n)[:n // 2]] = True
    for ch in range(3):
        v = np.array([117] * (n // 4) + [118] * (n // 4))
        rng.shuffle(v)
        u[dark, ch] = v
        u[~dark, ch] = rng.integers(225, 250, n - n // 2)
    rgb = ((u - 128) & 0xFF).astype(np.uint8).reshape(-1)
    ppm, quant, dec = str(tmp_path / "in.ppm"), str(tmp_path / "out.quant"), str(tmp_path / "dec.ppm")
    _write_ppm(ppm, rgb, S, S)
    r = subprocess.run([test_api, "compress", ppm, quant, dec, "1", "1", "1", "1"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    X, _ = oracle.tile(rgb, S, S, 1, 1)
    C_k, A_k, _ = oracle.lbg(X, 1, sum_mode=0)
    C_x = oracle.centroids(X, A_k, 2, sum_mode=1)
    # the dark cell sits next to a byte boundary: +/- 16 ulps of its exact-sum centroid straddle it
    c = C_x[np.argmin(C_x[:, 0]), 0]
    w = 16 * np.spacing(c)
    assert oracle.codebook_bytes(np.array([[c - w]]))[0, 0] != oracle.codebook_bytes(np.array([[c + w]]))[0, 0]
    expected = oracle.quant_file_bytes(oracle.codebook_bytes(C_k), A_k, 1, 1, S, S, 1, 1)
    assert open(quant, "rb").read() == expected
