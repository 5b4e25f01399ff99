"""quant_amd -- MI355X LBG vector-quantization engine (Python mirror of the C ABI).

The product is libqvq.so (quant_amd/lib), a C-ABI library of hand-written HIP kernels
for gfx950 (include/qvq.h).  This module binds it with ctypes and mirrors the
reference's quantizer plugin interface (include/Quantizer.hpp:8-20):

    getQuantizer(Quantizers.LBG).quantize(trainingSet, n, eps) -> (codebook, assigned, distortion)

There is no CPU fallback: every compute call goes to the GPU through libqvq.so and raises
QVQError when the library or the device is missing.
"""
import ctypes
import sys
import enum
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QVQ_LIB") or os.path.join(_HERE, "lib", "libqvq.so")   # QVQ_LIB: A/B builds (tools/)

NORMAL, SCALED, CIE1931 = 0, 1, 2   # enum class ColorSpaces (include/ColorSpace.hpp:6)


class QVQError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__("qvq status %d: %s" % (status, msg))
        self.status = status


class _Timings(ctypes.Structure):
    _fields_ = [("levels", ctypes.c_int), ("total_ms", ctypes.c_double),
                ("assign_ms", ctypes.c_double * 32), ("update_ms", ctypes.c_double * 32),
                ("other_ms", ctypes.c_double * 32), ("flagged", ctypes.c_uint64 * 32),
                ("host_ties", ctypes.c_uint64 * 32), ("wait_ms", ctypes.c_double * 32),
                ("tree_ms", ctypes.c_double * 32), ("kahan_redo", ctypes.c_int), ("tie_overflow", ctypes.c_int),
                ("kahan_relays", ctypes.c_int), ("mean_ms", ctypes.c_double)]


_lib = None
EXPORTED = ["qvq_create", "qvq_destroy", "qvq_last_error", "qvq_version", "qvq_set_images",
            "qvq_set_images_device", "qvq_set_synthetic", "qvq_set_vectors", "qvq_num_vectors",
            "qvq_dim", "qvq_lbg", "qvq_assign_device", "qvq_assign", "qvq_update", "qvq_update_kahan",
            "qvq_comm_unique_id", "qvq_comm_init", "qvq_set_timing", "qvq_get_timings", "qvq_host_kdtree_nn",
            "qvq_host_finalize", "qvq_host_row_terms", "qvq_decode", "qvq_decode_mse", "qvq_decode_device",
            "qvq_set_timeout", "qvq_host_wait_probe", "qvq_comm_init_host", "qvq_comm_info", "qvq_set_vectors_exact",
            "qvq_update_kahan_split", "qvq_host_pool_stress", "qvq_kdtree_device_check",
            "qvq_host_kdtree_image"]

COMM_NONE, COMM_RCCL, COMM_HOST = 0, 1, 2
# int fn(void *buf, uint64_t count, int dtype, void *user) (qvq.h, qvq_comm_init_host)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p)


def lib():
    """Load libqvq.so (built in-tree by __graft_entry__.build() / make -C quant_amd/csrc)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise QVQError(-1, "libqvq.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        P, u32, u64, i = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        sig = {
            "qvq_create": ([i, ctypes.POINTER(P)], i),
            "qvq_destroy": ([P], None),
            "qvq_last_error": ([P], ctypes.c_char_p),
            "qvq_version": ([], ctypes.c_char_p),
            "qvq_set_images": ([P, P, u32, u32, u32, u32, u32, i], i),
            "qvq_set_images_device": ([P, P, u32, u32, u32, u32, u32, i], i),
            "qvq_set_synthetic": ([P, u32, u64, u32, u32, u32, i], i),
            "qvq_set_vectors": ([P, P, u64, u32], i),
            "qvq_set_vectors_exact": ([P, P, u64, u32], i),
            "qvq_num_vectors": ([P], u64),
            "qvq_dim": ([P], u32),
            "qvq_lbg": ([P, u32, ctypes.c_double, P, P, P], i),
            "qvq_assign_device": ([P], P),
            "qvq_assign": ([P, P, u32, P], i),
            "qvq_update": ([P, P, u32, P, P], i),
            "qvq_update_kahan": ([P, P, u32, P], i),
            "qvq_update_kahan_split": ([P, P, u32, P, u32, P], i),
            "qvq_host_pool_stress": ([u32, u32, P], i),
            "qvq_comm_unique_id": ([P], i),
            "qvq_comm_init": ([P, i, i, P], i),
            "qvq_set_timing": ([P, i], i),
            "qvq_get_timings": ([P, ctypes.POINTER(_Timings)], i),
            "qvq_host_kdtree_nn": ([P, u32, u32, P, u64, P], i),
            "qvq_host_kdtree_image": ([P, u32, u32, P, u64, P], i),
            "qvq_kdtree_device_check": ([P, P, u32, u32, P, P], i),
            "qvq_host_finalize": ([P, P, P, u32, u32, i, P], i),
            "qvq_host_row_terms": ([P, u32, i, P, P], i),
            "qvq_decode": ([P, P, u32, P, u64, u32, u32, u32, u32, P], i),
            "qvq_decode_mse": ([P, P, u32, P, u64, u32, u32, u32, u32, P, P, P], i),
            "qvq_decode_device": ([P, P, u32, P, u64, u32, u32, u32, u32, P, P], i),
            "qvq_set_timeout": ([P, ctypes.c_double], i),
            "qvq_host_wait_probe": ([i, ctypes.c_double, P], i),
            "qvq_comm_init_host": ([P, i, i, ALLREDUCE_FN, P], i),
            "qvq_comm_info": ([P, ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(i)], i),
        }
        for name, (args, res) in sig.items():
            if os.environ.get("QVQ_LIB") and not hasattr(L, name):
                continue   # an older A/B build (tools/) without this entry point
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _check(st, ctx=None):
    if st != 0:
        msg = lib().qvq_last_error(ctx)
        raise QVQError(st, msg.decode() if msg else "")


def _torch_runtime_first():
    """PyTorch-ROCm wheels bundle their own HIP/HSA runtime next to the /opt/rocm one libqvq.so
    links.  When libqvq.so opens the device first, the bundled runtime's later device discovery
    fails ("No HIP GPUs are available"); the other order works.  So if torch is already loaded,
    let it open the device before the engine does."""
    torch = sys.modules.get("torch")
    if torch is not None:
        try:
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:   # no device for torch: the engine's own error says why
            pass


class Engine:
    """One qvq context: one GPU, one HIP stream, one resident training set."""

    def __init__(self, device=0):
        _torch_runtime_first()
        h = ctypes.c_void_p()
        L = lib()
        _check(L.qvq_create(device, ctypes.byref(h)))
        self._h = h
        self._L = L   # held by the engine: at interpreter shutdown the module globals may be gone

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            self._h = None
            self._L.qvq_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:   # noqa: BLE001  (interpreter shutdown: nothing left to report to)
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- training sets -------------------------------------------------------------------
    def set_images(self, rgb, n_images, xSize, ySize, bw, bh, colorspace=SCALED):
        rgb = np.ascontiguousarray(rgb, np.uint8)
        assert rgb.size == n_images * xSize * ySize * 3
        _check(lib().qvq_set_images(self._h, _p(rgb), n_images, xSize, ySize, bw, bh, colorspace), self._h)

    def set_images_device(self, ptr, n_images, xSize, ySize, bw, bh, colorspace=SCALED):
        _check(lib().qvq_set_images_device(self._h, ctypes.c_void_p(ptr), n_images, xSize, ySize, bw, bh,
                                           colorspace), self._h)

    def set_synthetic(self, S, seed0=0x5EED, n_images=1, bw=2, bh=2, colorspace=SCALED):
        _check(lib().qvq_set_synthetic(self._h, S, seed0, n_images, bw, bh, colorspace), self._h)

    def set_vectors(self, X, exact=False):
        """fp64 training set N x dim.  Byte-image values (NORMAL/SCALED) take the fast path; any
        other data -- or exact=True -- the exact mode (the reference's Kahan arithmetic, qvq.h)."""
        X = np.ascontiguousarray(X, np.float64)
        fn = lib().qvq_set_vectors_exact if exact else lib().qvq_set_vectors
        _check(fn(self._h, _p(X), X.shape[0], X.shape[1]), self._h)

    @property
    def n(self):
        return int(lib().qvq_num_vectors(self._h))

    @property
    def dim(self):
        return int(lib().qvq_dim(self._h))

    # -- hot path ------------------------------------------------------------------------
    def lbg(self, bits, eps=1e-6, want_assign=True, out=None):
        """Split-LBG to 2**bits code vectors: (codebook, indices or None, distortion).
        out: optional (C, d) float64 arrays of shapes (2**bits, dim) and (1,) to fill instead of
        allocating (repeated calls, e.g. bench.py)."""
        K = 1 << bits
        if out is None:
            C, d = np.empty((K, self.dim), np.float64), np.zeros(1, np.float64)
        else:
            C, d = out
            assert C.shape == (K, self.dim) and C.dtype == np.float64 and C.flags.c_contiguous
            assert d.shape == (1,) and d.dtype == np.float64
        A = np.empty(self.n, np.uint32) if want_assign else None
        _check(lib().qvq_lbg(self._h, bits, eps, _p(C), _p(A) if want_assign else None, _p(d)), self._h)
        return C, A, float(d[0])

    def assign(self, C):
        C = np.ascontiguousarray(C, np.float64)
        A = np.empty(self.n, np.uint32)
        _check(lib().qvq_assign(self._h, _p(C), C.shape[0], _p(A)), self._h)
        return A

    def update(self, A, K):
        A = np.ascontiguousarray(A, np.uint32)
        C = np.empty((K, self.dim), np.float64)
        cnt = np.empty(K, np.uint64)
        _check(lib().qvq_update(self._h, _p(A), K, _p(C), _p(cnt)), self._h)
        return C, cnt

    def update_kahan(self, A, K):
        """The reference's centroid bits (Kahan sums in row order, src/Quantizer.cpp:59-87)."""
        A = np.ascontiguousarray(A, np.uint32)
        C = np.empty((K, self.dim), np.float64)
        _check(lib().qvq_update_kahan(self._h, _p(A), K, _p(C)), self._h)
        return C

    def update_kahan_split(self, A, K, splits):
        """update_kahan with the rows cut into virtual ranks at splits (0 .. n): the several-rank
        chained evaluation run rank after rank on this device (test entry)."""
        A = np.ascontiguousarray(A, np.uint32)
        sp = np.ascontiguousarray(splits, np.uint64)
        C = np.empty((K, self.dim), np.float64)
        _check(lib().qvq_update_kahan_split(self._h, _p(A), K, _p(sp), sp.size - 1, _p(C)), self._h)
        return C

    def assign_device_ptr(self):
        return lib().qvq_assign_device(self._h)

    def kdtree_device_check(self, C):
        """The reference kd-tree of C (K x D) built on the device against the host's, node for node:
        (result, [launch ms, phase-1 ms, phase-2 ms, images ms], first difference); result 0 equal,
        1 different, 2 the build gave up."""
        C = np.ascontiguousarray(C, np.float64)
        ms = np.zeros(4, np.float64)
        res = np.zeros(1, np.uint32)
        _check(lib().qvq_kdtree_device_check(self._h, _p(C), C.shape[0], C.shape[1], _p(ms), _p(res)), self._h)
        why = lib().qvq_last_error(self._h).decode() if res[0] == 1 else ""
        return int(res[0]), [round(float(x), 4) for x in ms], why

    def set_timing(self, level=-1):
        """HIP events around the search of every level (-1), none (-2) or level+1 only."""
        _check(lib().qvq_set_timing(self._h, int(level)), self._h)

    def level_timing(self, level):
        """(search ms, update ms, flagged rows over all levels) of the last lbg, without
        building the full timings() dict (bench.py reads this once per step)."""
        t = getattr(self, "_tm", None)
        if t is None:
            t = self._tm = _Timings()
        _check(lib().qvq_get_timings(self._h, ctypes.byref(t)), self._h)
        return t.assign_ms[level], t.update_ms[level], sum(t.flagged[:max(t.levels, 1)])

    def timings(self):
        t = _Timings()
        _check(lib().qvq_get_timings(self._h, ctypes.byref(t)), self._h)
        L = t.levels
        return {"levels": L, "total_ms": t.total_ms,
                "assign_ms": list(t.assign_ms[:max(L, 1)]), "update_ms": list(t.update_ms[:max(L, 1)]),
                "other_ms": list(t.other_ms[:max(L, 1)]),
                "flagged": list(t.flagged[:max(L, 1)]), "host_ties": list(t.host_ties[:max(L, 1)]),
                "wait_ms": list(t.wait_ms[:max(L, 1)]), "tree_ms": list(t.tree_ms[:max(L, 1)]),
                "kahan_redo": t.kahan_redo, "tie_overflow": t.tie_overflow, "kahan_relays": t.kahan_relays,
                "mean_ms": t.mean_ms}

    # -- multi-GPU -----------------------------------------------------------------------
    def decode(self, cb_bytes, A, xSize, ySize, bw, bh):
        """CompressedImage::decompress (src/Compressor.cpp:156-165) on the device: codebook bytes
        (K x bw*bh*3 u8) and block indices -> xSize*ySize*3 raster (u8)."""
        cb = np.ascontiguousarray(cb_bytes, dtype=np.uint8).reshape(-1, bw * bh * 3)
        A = np.ascontiguousarray(A, dtype=np.uint32).ravel()
        out = np.empty(xSize * ySize * 3, dtype=np.uint8)
        _check(lib().qvq_decode(self._h, _p(cb), cb.shape[0], _p(A), A.size, xSize, ySize, bw, bh, _p(out)), self._h)
        return out

    def decode_mse(self, cb_bytes, A, xSize, ySize, bw, bh, orig, want_image=True):
        """Decode plus the raport's distortion (src/Compressor.cpp:133-146): mean squared
        difference of the signed bytes of orig and the decoded raster, in the same device pass.
        Returns (raster or None, mse)."""
        cb = np.ascontiguousarray(cb_bytes, dtype=np.uint8).reshape(-1, bw * bh * 3)
        A = np.ascontiguousarray(A, dtype=np.uint32).ravel()
        orig = np.ascontiguousarray(orig, dtype=np.uint8).ravel()
        assert orig.size == xSize * ySize * 3
        out = np.empty(xSize * ySize * 3, dtype=np.uint8) if want_image else None
        mse = ctypes.c_double()
        _check(lib().qvq_decode_mse(self._h, _p(cb), cb.shape[0], _p(A), A.size, xSize, ySize, bw, bh,
                                    _p(out) if want_image else None, _p(orig), ctypes.byref(mse)), self._h)
        return out, mse.value

    def set_timeout(self, seconds):
        """Bound of every host wait on the engine's stream (QVQ_ECOMM / QVQ_EDEVICE past it)."""
        _check(lib().qvq_set_timeout(self._h, float(seconds)), self._h)

    def decode_device(self, cb_ptr, K, a_ptr, nblocks, xSize, ySize, bw, bh, rgb_ptr, stream=None):
        """Device-pointer decode on `stream` (a hipStream_t handle; None or 0 = the legacy null
        stream, ordered after the caller's work on blocking streams)."""
        _check(lib().qvq_decode_device(self._h, cb_ptr, K, a_ptr, nblocks, xSize, ySize, bw, bh, rgb_ptr, stream),
               self._h)

    @staticmethod
    def comm_unique_id():
        buf = (ctypes.c_uint8 * 128)()
        _check(lib().qvq_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, nranks, rank, uid):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        _check(lib().qvq_comm_init(self._h, nranks, rank, buf), self._h)

    def comm_init_host(self, nranks, rank, allreduce):
        """Test-only communicator (qvq_comm_init_host): allreduce(arr) must replace the numpy
        array arr (uint64 or float64) in place by its sum over the ranks, e.g. through
        torch.distributed's gloo backend.  Lets several processes share one GPU."""
        def cb(ptr, count, dtype, user):
            try:
                ct = ctypes.c_uint64 if dtype == 0 else ctypes.c_double
                arr = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), shape=(count,))
                allreduce(arr)
                return 0
            except Exception:   # noqa: BLE001  (no exception may cross the C ABI)
                import traceback
                traceback.print_exc()
                return 1
        self._ar_cb = ALLREDUCE_FN(cb)   # kept alive with the engine
        _check(lib().qvq_comm_init_host(self._h, nranks, rank, self._ar_cb, None), self._h)

    def comm_info(self):
        """(nranks, rank, kind) of the joined communicator; kind COMM_NONE/COMM_RCCL/COMM_HOST."""
        n, r, k = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(lib().qvq_comm_info(self._h, ctypes.byref(n), ctypes.byref(r), ctypes.byref(k)), self._h)
        return n.value, r.value, k.value


# -- host-only helpers (no GPU) ------------------------------------------------------------
def host_kdtree_nn(C, Q):
    C = np.ascontiguousarray(C, np.float64)
    Q = np.ascontiguousarray(Q, np.float64)
    out = np.empty(Q.shape[0], np.uint32)
    _check(lib().qvq_host_kdtree_nn(_p(C), C.shape[0], C.shape[1], _p(Q), Q.shape[0], _p(out)))
    return out


# KdbNode (kdtree_dev.hpp) and the image layout of qvq_host_kdtree_image
KDB_NODE = np.dtype([("child1", "<i4"), ("child2", "<i4"), ("left", "<u4"), ("right", "<u4"), ("divfeat", "<i4"),
                     ("depth", "<u4"), ("divlow", "<f8"), ("divhigh", "<f8"), ("cutval", "<f8"),
                     ("split_val", "<f8"), ("spread_gap", "<f8"), ("cand", "<u8")])
KDB_HEADER_BYTES = 64


def host_kdtree_image(C):
    """The host build of C's kd-tree (RefKDTree) as arrays: (nodes [n] KDB_NODE breadth first,
    lo [n, D], hi [n, D] point boxes, vind [K], depth)."""
    C = np.ascontiguousarray(C, np.float64)
    K, D = C.shape
    need = ctypes.c_uint64()
    lib().qvq_host_kdtree_image(_p(C), K, D, None, 0, ctypes.byref(need))
    img = np.zeros(need.value, np.uint8)
    _check(lib().qvq_host_kdtree_image(_p(C), K, D, _p(img), img.size, ctypes.byref(need)))
    n_nodes, depth = (int(x) for x in img[:8].view("<u4"))
    off = KDB_HEADER_BYTES
    nodes = img[off:off + 2 * K * KDB_NODE.itemsize].view(KDB_NODE)[:n_nodes]
    off += 2 * K * KDB_NODE.itemsize
    boxes = img[off:off + 2 * K * 2 * D * 8].view("<f8").reshape(2 * K, 2, D)[:n_nodes]
    off += 2 * K * 2 * D * 8
    vind = img[off:off + 4 * K].view("<u4")
    return nodes, boxes[:, 0], boxes[:, 1], vind.copy(), depth


def host_wait_probe(scenario, timeout_s):
    """The engine's bounded-wait policy under scripted probes (qvq.h): (status, seconds)."""
    el = ctypes.c_double()
    st = lib().qvq_host_wait_probe(int(scenario), float(timeout_s), ctypes.byref(el))
    return st, el.value


def host_pool_stress(rounds, maxn):
    """The certificate's thread pool under jobs of changing width (qvq.h): slots run != once."""
    bad = ctypes.c_uint64()
    _check(lib().qvq_host_pool_stress(int(rounds), int(maxn), ctypes.byref(bad)))
    return bad.value


def host_finalize(hi, lo, cnt, colorspace=SCALED):
    hi = np.ascontiguousarray(hi, np.uint64)
    lo = np.ascontiguousarray(lo, np.uint64)
    cnt = np.ascontiguousarray(cnt, np.uint64)
    K, D = hi.shape
    C = np.empty((K, D), np.float64)
    _check(lib().qvq_host_finalize(_p(hi), _p(lo), _p(cnt), K, D, colorspace, _p(C)))
    return C


def host_row_terms(codes, colorspace=SCALED):
    """(hi, lo) exact-sum terms of each byte code, shape like codes (uint64)."""
    codes = np.ascontiguousarray(codes, np.uint8)
    flat = codes.reshape(-1)
    hi = np.empty(flat.size, np.uint64)
    lo = np.empty(flat.size, np.uint64)
    _check(lib().qvq_host_row_terms(_p(flat), flat.size, colorspace, _p(hi), _p(lo)))
    return hi.reshape(codes.shape), lo.reshape(codes.shape)


# -- the reference's plugin interface (include/Quantizer.hpp:8-20) ---------------------------
class Quantizers(enum.IntEnum):
    LBG = 0
    MEDIAN_CUT = 1
    LBG_MEDIAN_CUT = 2
    ABC = 3


class AbstractQuantizer:
    def quantize(self, trainingSet, n, eps):
        raise NotImplementedError


class LBGQuantizer(AbstractQuantizer):
    """LBGQuantizer (src/Quantizer.cpp:119-144) on the MI355X engine."""

    def __init__(self, device=0):
        self._device = device
        self._engine = None

    def quantize(self, trainingSet, n, eps):
        if self._engine is None:
            self._engine = Engine(self._device)
        self._engine.set_vectors(np.asarray(trainingSet, np.float64))
        return self._engine.lbg(int(n), eps)


def getQuantizer(q):
    """src/Quantizer.cpp:146-155: only LBG exists; other enumerators give None."""
    return LBGQuantizer() if Quantizers(q) == Quantizers.LBG else None
