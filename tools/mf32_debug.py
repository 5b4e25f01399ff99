"""Debug: the duplicate-tie case of test_assign_ties_and_duplicates, old vs new search."""
import os, subprocess, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
if len(sys.argv) == 1:
    for v in ("0", "1"):
        for kd in ("device", "host"):
            env = dict(os.environ, QVQ_MF32=v, QVQ_KDTREE=kd)
            subprocess.run([sys.executable, __file__, "run"], env=env, check=True)
    sys.exit(0)
import quant_amd
from oracle import oracle
rng = np.random.default_rng(7)
X, _ = oracle.tile(oracle.gen_image(128), 128, 128, 2, 2)
base = X[rng.choice(len(X), 40, replace=False)]
C = np.concatenate([base * (1 + 0.2), base * (1 - 0.2), np.zeros((8, 12)), base[:4], base[:4]])
ref = oracle.kdtree_nn(C, X)
with quant_amd.Engine(0) as eng:
    eng.set_vectors(X)
    A = eng.assign(C)
    t = eng.timings()
bad = np.nonzero(A != ref)[0]
d = ((X[:, None, :] - C[None, :, :]) ** 2).sum(-1)
info = []
for r in bad[:5]:
    o = np.argsort(d[r])[:4]
    info.append({"row": int(r), "got": int(A[r]), "ref": int(ref[r]), "near": [(int(k), float(d[r, k])) for k in o]})
print(json.dumps({"mf32": os.environ.get("QVQ_MF32"), "kd": os.environ.get("QVQ_KDTREE"), "nbad": len(bad),
                  "flagged": t["flagged"], "host_ties": t["host_ties"], "bad": info}), flush=True)
