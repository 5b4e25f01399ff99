import sys, numpy as np
sys.path.insert(0, "/root/repo")
import quant_amd
eng = quant_amd.Engine(0)
for bw, bits in ((4, 11), (2, 9)):
    eng.set_synthetic(4096, 0x5EED, 1, bw, bw)
    C, A, d = eng.lbg(bits, want_assign=False)
    np.save(f"/root/repo/gpurun_out/cb_{bw}_{bits}.npy", C)
    print(C.shape, (np.abs(C).sum(1) == 0).sum(), "zero rows")
