import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libqvq.so)")
    config.addinivalue_line("markers", "slow: long CPU oracle runs")


def load_png_rgb(name):
    """Reference image fixture -> (raster bytes, xSize, ySize) as RGBImage reads a P6 file."""
    from PIL import Image
    im = Image.open(os.path.join(GOLDEN, name)).convert("RGB")
    w, h = im.size
    return np.frombuffer(im.tobytes(), np.uint8).copy(), w, h


def reference_lbg(X, bits):
    """The oracle's reference rule (Kahan centroids, sum_mode 0): its indices A_k, codebook C_k,
    distortion d_k, and C_e, the engine's codebook for those indices (the exact-sum centroids
    of the final cells, its documented centroid rule: within 1e-12 of C_k)."""
    from oracle import oracle
    C_k, A_k, d_k = oracle.lbg(X, bits, sum_mode=0)
    C_e = oracle.centroids(X, A_k, 1 << bits, sum_mode=1)
    return C_e, A_k, d_k, C_k


@pytest.fixture(scope="session")
def engine():
    import torch   # noqa: F401  (torch's bundled HIP runtime opens the device first: quant_amd.Engine)
    import quant_amd
    eng = quant_amd.Engine(0)
    yield eng
    eng.close()
