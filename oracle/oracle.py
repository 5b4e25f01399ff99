"""ctypes binding of the C oracle (lbg_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the parity checker.  The product never imports this module.
"""
import ctypes
import hashlib
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")

NORMAL, SCALED = 0, 1
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        sz = ctypes.c_size_t
        i = ctypes.c_int
        _lib.orc_lbg.argtypes = [P, sz, i, i, ctypes.c_double, i, i, P, P, P, P, P]
        _lib.orc_lbg.restype = i
        _lib.orc_tile.argtypes = [P, i, i, i, i, i, P, P, ctypes.c_uint8]
        _lib.orc_untile.argtypes = [P, i, i, i, i, P]
        _lib.orc_num_blocks.argtypes = [i, i, i, i]
        _lib.orc_num_blocks.restype = sz
        _lib.orc_gen_image.argtypes = [ctypes.c_uint32, ctypes.c_uint64, P]
        _lib.orc_lut.argtypes = [i, P]
        _lib.orc_codebook_bytes.argtypes = [P, sz, i, i, P]
        _lib.orc_kdtree_nn.argtypes = [P, sz, i, P, sz, P]
        _lib.orc_bruteforce.argtypes = [P, sz, i, P, sz, P, P]
        _lib.orc_centroids.argtypes = [P, sz, i, P, sz, i, P]
        _lib.orc_centroids.restype = i
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def sha16(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def gen_image(S, seed=0x5EED):
    """Synthetic S x S RGB raster, shape (S*S*3,) uint8."""
    out = np.empty(S * S * 3, np.uint8)
    lib().orc_gen_image(S, seed, _p(out))
    return out


def read_ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(maxsplit=4)
    assert parts[0] == b"P6"
    xs, ys = int(parts[1]), int(parts[2])
    # header is "P6 <ws> x <ws> y <ws> 255" + one whitespace byte (src/RGBImage.cpp:6-24)
    hdr = data.index(parts[3]) + len(parts[3]) + 1
    return np.frombuffer(data[hdr:hdr + xs * ys * 3], np.uint8).copy(), xs, ys


def lut(cs=SCALED):
    out = np.empty(256, np.float64)
    lib().orc_lut(cs, _p(out))
    return out


def tile(rgb, xs, ys, bw, bh, cs=SCALED, pad_code=128):
    """getBlocksAsVectorsFromImage: returns (X [N, D] float64, codes [N, D] uint8)."""
    n = lib().orc_num_blocks(xs, ys, bw, bh)
    D = 3 * bw * bh
    X = np.empty((n, D), np.float64)
    codes = np.empty((n, D), np.uint8)
    rgb = np.ascontiguousarray(rgb, np.uint8)
    lib().orc_tile(_p(rgb), xs, ys, bw, bh, cs, _p(X), _p(codes), pad_code)
    return X, codes


def untile(blocks, xs, ys, bw, bh):
    blocks = np.ascontiguousarray(blocks, np.uint8)
    out = np.empty(xs * ys * 3, np.uint8)
    lib().orc_untile(_p(blocks), xs, ys, bw, bh, _p(out))
    return out


def lbg(X, bits, eps=1e-6, sum_mode=0, threads=0, dump=False):
    """LBGQuantizer::quantize restated.  sum_mode 0 = Kahan (reference), 1 = exact sums.
    Returns (C [2^bits, D], A [N] uint32, distortion[, C_split list, A list])."""
    X = np.ascontiguousarray(X, np.float64)
    N, D = X.shape
    K = 1 << bits
    C = np.empty((K, D), np.float64)
    A = np.empty(N, np.uint32)
    dist = np.zeros(1, np.float64)
    Cs = np.empty(max(1, (2 * K - 2) * D), np.float64) if dump else None
    As = np.empty(max(1, bits * N), np.uint32) if dump else None
    rc = lib().orc_lbg(_p(X), N, D, bits, eps, sum_mode, threads, _p(C), _p(A), _p(dist),
                       _p(Cs) if dump else None, _p(As) if dump else None)
    if rc != 0:
        raise RuntimeError("orc_lbg failed: %d" % rc)
    if not dump:
        return C, A, float(dist[0])
    splits, assigns, off = [], [], 0
    for lvl in range(1, bits + 1):
        k = 1 << lvl
        splits.append(Cs[off:off + k * D].reshape(k, D).copy())
        assigns.append(As[(lvl - 1) * N:lvl * N].copy())
        off += k * D
    return C, A, float(dist[0]), splits, assigns


def kdtree_nn(C, Q):
    C = np.ascontiguousarray(C, np.float64)
    Q = np.ascontiguousarray(Q, np.float64)
    out = np.empty(Q.shape[0], np.uint32)
    lib().orc_kdtree_nn(_p(C), C.shape[0], C.shape[1], _p(Q), Q.shape[0], _p(out))
    return out


def bruteforce(C, Q):
    C = np.ascontiguousarray(C, np.float64)
    Q = np.ascontiguousarray(Q, np.float64)
    out = np.empty(Q.shape[0], np.uint32)
    nt = np.empty(Q.shape[0], np.uint32)
    lib().orc_bruteforce(_p(C), C.shape[0], C.shape[1], _p(Q), Q.shape[0], _p(out), _p(nt))
    return out, nt


def centroids(X, A, K, sum_mode=1):
    X = np.ascontiguousarray(X, np.float64)
    A = np.ascontiguousarray(A, np.uint32)
    C = np.empty((K, X.shape[1]), np.float64)
    if lib().orc_centroids(_p(X), X.shape[0], X.shape[1], _p(A), K, sum_mode, _p(C)) != 0:
        raise RuntimeError("orc_centroids failed")
    return C


def codebook_bytes(C, cs=SCALED):
    C = np.ascontiguousarray(C, np.float64)
    out = np.empty(C.shape, np.uint8)
    lib().orc_codebook_bytes(_p(C), C.shape[0], C.shape[1], cs, _p(out))
    return out


def quant_file_bytes(cb_bytes, A, bits, cs, xs, ys, bw, bh):
    """CompressedImage::saveToFile (src/Compressor.cpp:191-224) restated: ASCII header
    'bits colorSpace count xSize ySize bw bh\\n', 2^bits x (bw*bh*3) codebook bytes, then
    count indices of ceil(bits/8) little-endian bytes.  colorSpace is written as the real
    enum value (the reference leaves CompressedImage::colorSpace unset)."""
    A = np.asarray(A, np.uint64)
    nb = (bits + 7) // 8
    hdr = ("%d %d %d %d %d %d %d\n" % (bits, cs, len(A), xs, ys, bw, bh)).encode()
    idx = np.stack([((A >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.uint8) for b in range(nb)], axis=1)
    return hdr + np.ascontiguousarray(cb_bytes, np.uint8).tobytes() + idx.tobytes()


def decode(cb_bytes, A, xs, ys, bw, bh):
    """CompressedImage::decompress (src/Compressor.cpp:156-165): gather + untile."""
    blocks = np.ascontiguousarray(cb_bytes, np.uint8)[np.asarray(A, np.int64)]
    return untile(blocks, xs, ys, bw, bh)


def raport_distortion(rgb, dec):
    """src/Compressor.cpp:133-144: mean squared difference of the signed bytes."""
    a = np.asarray(rgb, np.uint8).view(np.int8).astype(np.float64)
    b = np.asarray(dec, np.uint8).view(np.int8).astype(np.float64)
    return float(np.mean((a - b) ** 2))
