"""Wide MFMA search vs the VALU search on the same codebooks (diagnostics)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import quant_amd

eng = quant_amd.Engine(0)
for (S, bw, bh, K) in [(256, 2, 3, 32), (256, 2, 3, 64), (256, 1, 1, 64), (256, 4, 4, 64), (512, 4, 4, 1024),
                       (256, 2, 1, 128)]:
    eng.set_synthetic(S, 0x5EED, 1, bw, bh)
    os.environ["QVQ_SEARCH"] = "valu"
    C, A0, _ = eng.lbg(int(np.log2(K)))
    Av = eng.assign(C)
    os.environ["QVQ_SEARCH"] = "mfma"
    Aw = eng.assign(C)
    tm = eng.timings()
    bad = np.nonzero(Av != Aw)[0]
    print(f"S={S} {bw}x{bh} K={K}: mismatches {len(bad)} of {len(Av)}; flagged {tm['flagged'][:2]}", flush=True)
    if len(bad):
        i = bad[:5]
        print("   rows", i.tolist(), "valu", Av[i].tolist(), "wide", Aw[i].tolist(), flush=True)
