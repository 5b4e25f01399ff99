"""Time the decode gather (qvq_decode_device) at C3 size: 4096^2 raster, 2x2 blocks, K=1024.
Algorithmic bytes per launch = 4 B/block index + 3 B/pixel written (codebook 12 KB stays in L2)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import quant_amd  # noqa: E402

xs = ys = 4096
K, steps = 1024, 50
rng = np.random.default_rng(1)
cb = torch.from_numpy(rng.integers(0, 256, (K, 12), dtype=np.uint8)).cuda()
nb = (xs // 2) * (ys // 2)
A = torch.from_numpy(rng.integers(0, K, nb, dtype=np.uint32).view(np.int32)).cuda()
out = torch.empty(xs * ys * 3, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream()
with quant_amd.Engine(0) as e:
    run = lambda: e.decode_device(cb.data_ptr(), K, A.data_ptr(), nb, xs, ys, 2, 2, out.data_ptr(), s.cuda_stream)
    for _ in range(5):
        run()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record(s)
    for _ in range(steps):
        run()
    t1.record(s)
    torch.cuda.synchronize()
ms = t0.elapsed_time(t1) / steps
alg = nb * 4 + xs * ys * 3
print(json.dumps({"kernel": "qvq::decode_kernel", "ms_per_call_incl_sync": ms, "alg_bytes": alg,
                  "GBps_incl_sync": alg / ms / 1e6}))
