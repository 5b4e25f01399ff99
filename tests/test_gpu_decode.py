"""GPU parity of the decode gather (qvq_decode / qvq_decode_device) against the oracle's
CompressedImage::decompress restatement (oracle.decode -> orc_untile, reference
src/Compressor.cpp:156-165 and :64-85).  Bar: bit-exact bytes."""
import numpy as np
import pytest

from conftest import load_png_rgb
from oracle import oracle

pytestmark = pytest.mark.gpu


def _rand_case(rng, xs, ys, bw, bh, K):
    D = bw * bh * 3
    cb = rng.integers(0, 256, size=(K, D), dtype=np.uint8)
    nb = -(-xs // bw) * -(-ys // bh)
    A = rng.integers(0, K, size=nb, dtype=np.uint32)
    return cb, A


@pytest.mark.parametrize("xs,ys,bw,bh,K", [
    (64, 64, 2, 2, 16), (510, 383, 2, 2, 64), (383, 510, 3, 5, 32), (7, 5, 4, 4, 8),
    (1, 1, 2, 2, 2), (3, 1, 1, 4, 4), (2, 3, 5, 7, 4), (129, 97, 4, 4, 1024), (33, 65, 1, 1, 256),
    # heights 1/2/4/8 without overhang, ys % 512 == 0: the LDS-staged coalesced store path
    (65, 512, 3, 1, 64), (130, 1024, 2, 2, 700), (7, 512, 4, 4, 33), (9, 1536, 2, 8, 5),
])
def test_decode_random_vs_oracle(engine, xs, ys, bw, bh, K):
    rng = np.random.default_rng(xs * 1000 + ys * 10 + bw)
    cb, A = _rand_case(rng, xs, ys, bw, bh, K)
    got = engine.decode(cb, A, xs, ys, bw, bh)
    want = oracle.decode(cb, A, xs, ys, bw, bh).ravel()
    np.testing.assert_array_equal(got, want)


def test_decode_after_lbg_matches_oracle(engine):
    rgb, xs, ys = load_png_rgb("t.png")   # 510 x 383: odd height wraps a block column
    engine.set_images(rgb, 1, xs, ys, 2, 2)
    C, A, _ = engine.lbg(6)
    cb = oracle.codebook_bytes(C)
    got = engine.decode(cb, A, xs, ys, 2, 2)
    np.testing.assert_array_equal(got, oracle.decode(cb, A, xs, ys, 2, 2).ravel())


def test_decode_rejects_bad_index(engine):
    import quant_amd
    cb = np.zeros((4, 12), np.uint8)
    A = np.array([0, 1, 2, 4], np.uint32)
    with pytest.raises(quant_amd.QVQError):
        engine.decode(cb, A, 4, 4, 2, 2)
    with pytest.raises(quant_amd.QVQError):
        engine.decode(cb, A[:3], 4, 4, 2, 2)


def test_decode_device_c3_checksum(engine):
    # BASELINE C3 size (4096^2, 2x2, K=1024) through device pointers; the oracle decodes the
    # same inputs on the host (a few hundred ms) and the rasters must match byte for byte.
    import torch
    xs = ys = 4096
    rng = np.random.default_rng(7)
    cb, A = _rand_case(rng, xs, ys, 2, 2, 1024)
    d_cb = torch.from_numpy(cb).cuda()
    d_A = torch.from_numpy(A.view(np.int32)).cuda()
    d_rgb = torch.empty(xs * ys * 3, dtype=torch.uint8, device="cuda")
    engine.decode_device(d_cb.data_ptr(), 1024, d_A.data_ptr(), A.size, xs, ys, 2, 2, d_rgb.data_ptr(),
                         torch.cuda.current_stream().cuda_stream)
    np.testing.assert_array_equal(d_rgb.cpu().numpy(), oracle.decode(cb, A, xs, ys, 2, 2).ravel())


@pytest.mark.parametrize("xs,ys,bw,bh", [(510, 383, 2, 2), (256, 256, 2, 2), (383, 512, 4, 4), (33, 65, 1, 1),
                                         (130, 1024, 2, 2), (17, 512, 1, 1), (5, 512, 3, 8)])
def test_decode_mse_matches_raport(engine, xs, ys, bw, bh):
    """qvq_decode_mse: the raport's distortion (src/Compressor.cpp:133-146, signed bytes) from
    the same device pass as the decoded raster."""
    rng = np.random.default_rng(xs + ys)
    cb, A = _rand_case(rng, xs, ys, bw, bh, 64)
    orig = rng.integers(0, 256, size=xs * ys * 3, dtype=np.uint8)
    img, mse = engine.decode_mse(cb, A, xs, ys, bw, bh, orig)
    want = oracle.decode(cb, A, xs, ys, bw, bh).ravel()
    np.testing.assert_array_equal(img, want)
    assert mse == oracle.raport_distortion(orig, want)   # integer sum / count: exact
    _, mse2 = engine.decode_mse(cb, A, xs, ys, bw, bh, orig, want_image=False)
    assert mse2 == mse


@pytest.mark.parametrize("which", ["torch_stream", "null_stream"])
def test_decode_device_orders_after_caller_stream(engine, which):
    """The decode launches on the caller's stream (0 = the legacy null stream), so indices a
    device op writes just before the call are the ones decoded."""
    import torch
    xs = ys = 1024
    rng = np.random.default_rng(3)
    cb, A = _rand_case(rng, xs, ys, 2, 2, 256)
    d_cb = torch.from_numpy(cb).cuda()
    src = torch.from_numpy(A.view(np.int32)).cuda()
    d_A = torch.zeros_like(src)
    d_rgb = torch.empty(xs * ys * 3, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    if which == "torch_stream":
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            torch.cuda._sleep(2_000_000)      # keep the stream busy so an unordered read sees zeros
            d_A.copy_(src)
        handle = s.cuda_stream
    else:
        torch.cuda._sleep(2_000_000)          # legacy default stream
        d_A.copy_(src)
        handle = 0
    engine.decode_device(d_cb.data_ptr(), 256, d_A.data_ptr(), A.size, xs, ys, 2, 2, d_rgb.data_ptr(), handle)
    np.testing.assert_array_equal(d_rgb.cpu().numpy(), oracle.decode(cb, A, xs, ys, 2, 2).ravel())
