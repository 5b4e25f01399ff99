"""The device kd build's plane split (k_kdbuild.hip) is nanoflann 1.2.3's two serial Hoare passes
(nanoflann.hpp:1159-1186, kdtree.cpp plane_split) restated with prefix counts: pass 1 over [0, n)
leaves lim1 = #(v < cut) and swaps the k-th element >= cut in [0, lim1) (counted from the left)
with the k-th element < cut in [lim1, n) (counted from the right); pass 2 does the same over
[lim1, n) with <=.  This checks that model against the serial passes on tie-heavy random arrays,
position for position (the GPU tests then check the kernel against the host tree node for node)."""
import numpy as np


def serial_passes(v, cut):
    """kdtree.cpp plane_split on an index array over values v (the reference's loops)."""
    ind = list(range(len(v)))
    n = len(v)
    left, right = 0, n - 1
    while True:
        while left <= right and v[ind[left]] < cut:
            left += 1
        while right and left <= right and v[ind[right]] >= cut:
            right -= 1
        if left > right or not right:
            break
        ind[left], ind[right] = ind[right], ind[left]
        left += 1
        right -= 1
    lim1 = left
    right = n - 1
    while True:
        while left <= right and v[ind[left]] <= cut:
            left += 1
        while right and left <= right and v[ind[right]] > cut:
            right -= 1
        if left > right or not right:
            break
        ind[left], ind[right] = ind[right], ind[left]
        left += 1
        right -= 1
    return ind, lim1, left


def paired_passes(v, cut):
    """The device form: each pass pairs misfits and partners by their ranks (prefix counts)."""
    ind = np.arange(len(v))
    vals = np.asarray(v, dtype=np.float64)
    lims = []
    start = 0
    for strict in (True, False):
        cur = vals[ind]
        fits = cur < cut if strict else cur <= cut
        fits[:start] = False
        lim = start + int(fits[start:].sum())
        pos = np.arange(len(v))
        misfit = (pos >= start) & (pos < lim) & ~fits   # from the left, in order
        partner = (pos >= lim) & fits                   # from the right, in order
        m = np.nonzero(misfit)[0]
        p = np.nonzero(partner)[0][::-1]
        assert len(m) == len(p)
        new = ind.copy()
        new[m], new[p] = ind[p], ind[m]
        ind = new
        lims.append(lim)
        start = lim
    return list(ind), lims[0], lims[1]


def test_pairing_matches_the_serial_passes():
    rng = np.random.default_rng(3)
    cases = 0
    for n in (11, 12, 13, 20, 64, 127, 128, 129, 500, 2048):
        for levels in (2, 3, 7, 50, 10 ** 6):
            for _ in range(6):
                v = rng.integers(0, levels, n).astype(np.float64)
                v[rng.random(n) < 0.3] = 0.0   # runs of duplicates (the zero code vectors)
                cand = [v.min(), v.max(), float(np.median(v)), float(v[rng.integers(n)]), v.mean()]
                for cut in cand:
                    a = serial_passes(v, cut)
                    b = paired_passes(v, cut)
                    assert a[1] == b[1] and a[2] == b[2], (n, levels, cut)
                    assert a[0] == b[0], (n, levels, cut)
                    cases += 1
    assert cases > 1000
