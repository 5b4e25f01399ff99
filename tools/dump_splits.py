"""Every level's split codebook of C3 (4096^2, 2x2, 10 bits) and C4 (4096^2, 4x4, 12 bits) from
the engine (lbg with 1..bits-1 levels; the next split is C * 1.2 | C * 0.8, src/Quantizer.cpp:134-138),
saved for the host analysis of the kd-tree shapes (tools/kd_shapes.py) and the device build tests.
usage: python tools/dump_splits.py OUT.npz"""
import sys
import numpy as np
sys.path.insert(0, "/root/repo")
import quant_amd


def splits(eng, bw, bits):
    eng.set_synthetic(4096, 0x5EED, 1, bw, bw)
    out = {}
    for L in range(1, bits):
        C, _, _ = eng.lbg(L, want_assign=False)
        out["b%d_L%d" % (bw, L + 1)] = np.concatenate([C * (1 + 0.2), C * (1 - 0.2)])
    return out


eng = quant_amd.Engine(0)
res = {}
res.update(splits(eng, 4, 12))
res.update(splits(eng, 2, 10))
np.savez_compressed(sys.argv[1], **res)
print({k: v.shape for k, v in res.items()})
