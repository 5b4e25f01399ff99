"""Device cost of the reference-bit (Kahan) centroids of a whole level (k_kahan.hip through
qvq_update_kahan), for the check of the last level: C3 (K=512 parent cells, D=12, 4.19M rows)
and C4 (K=2048 parent cells, D=48, 1.05M rows).  Run under rocprofv3 --kernel-trace."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import quant_amd  # noqa: E402

eng = quant_amd.Engine(0)
for S, bw, bits in ((4096, 2, 9), (4096, 4, 11)):
    eng.set_synthetic(S, 0x5EED, 1, bw, bw)
    C, A, d = eng.lbg(bits)
    K = 1 << bits
    for rep in range(4):
        t = time.perf_counter()
        Ck = eng.update_kahan(A, K)
        dt = time.perf_counter() - t
    print("S %d bw %d cells %d: update_kahan wall %.3f ms, max |Ck - C| %.3g" % (S, bw, K, dt * 1e3,
                                                                              float(np.max(np.abs(Ck - C)))), flush=True)
eng.close()
