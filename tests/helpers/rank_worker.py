"""One rank of the world-N GPU test (tests/test_gpu_multigpu.py): N of these processes share
GPU 0, exchange the per-level sums through the engine's test-only host communicator
(qvq_comm_init_host) over torch.distributed's gloo backend, and each runs qvq_lbg on its own
shard of the rows -- the sharded schedule of SURVEY.md 8(e) (reference loops
src/Quantizer.cpp:27-31 assign, :80-86 fix), executed for real.

    python rank_worker.py RANK WORLD RENDEZVOUS_FILE CASE OUT.npz
CASE: c2 -- the C2 image (512^2, 2x2) split into contiguous row ranges (qvq_set_vectors);
      c5 -- the reduced C5 batch (4 x 512^2 images, 2x2), whole images per rank (qvq_set_synthetic);
      corpus -- every case of tests/golden/kahan_divergent.json (inputs where the reference's
      Kahan centroid bits decide an index), rows split into contiguous ranges: per case the
      quantize (C{i}, A{i}, d{i}, redo{i}) and qvq_update_kahan of the local indices (K{i}: the
      reference's centroids over every rank's rows).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def shard(n, world, rank):
    return n * rank // world, n * (rank + 1) // world


def main():
    rank, world, rdv, case, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]
    import datetime
    import torch
    import torch.distributed as dist
    import quant_amd
    # a file rendezvous (no TCP store port picked ahead by the parent, which another process could
    # take first), and a bounded one: a rank that cannot join fails instead of waiting 30 minutes
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    dist.init_process_group("gloo", init_method="file://" + rdv, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))

    def allreduce(arr):
        t = torch.from_numpy(arr.view(np.int64) if arr.dtype == np.uint64 else arr)   # shares arr's memory
        dist.all_reduce(t)   # int64 sums wrap like the engine's u64 sums

    eng = quant_amd.Engine(0)
    eng.comm_init_host(world, rank, allreduce)
    if case == "c2":
        from oracle import oracle
        X, _ = oracle.tile(oracle.gen_image(512, 0x5EED), 512, 512, 2, 2)
        lo, hi = shard(X.shape[0], world, rank)
        eng.set_vectors(X[lo:hi])
    elif case == "c5":
        lo, hi = shard(4, world, rank)
        eng.set_synthetic(512, 0x5EED + lo, hi - lo, 2, 2)
    elif case == "corpus":
        import json
        from oracle import oracle
        sys.path.insert(0, os.path.join(ROOT, "tests", "helpers"))
        from kahan_env_worker import make
        corpus = json.load(open(os.path.join(ROOT, "tests", "golden", "kahan_divergent.json")))
        res = {}
        for i, c in enumerate(corpus["noise_seeds"] + corpus["found"]):
            X, _ = oracle.tile(make(c), c["side"], c["side"], c["bw"], c["bh"])
            lo, hi = shard(X.shape[0], world, rank)
            eng.set_vectors(X[lo:hi])
            C, A, d = eng.lbg(c["bits"])
            tm = eng.timings()
            res.update({"C%d" % i: C, "A%d" % i: A, "d%d" % i: np.array([d]), "redo%d" % i: np.array([tm["kahan_redo"]]),
                        "relays%d" % i: np.array([tm["kahan_relays"]]),
                        "K%d" % i: eng.update_kahan(A, 1 << c["bits"])})
        np.savez(out, info=np.array(eng.comm_info()), **res)
        eng.close()
        dist.destroy_process_group()
        return
    else:
        raise SystemExit("unknown case " + case)
    C, A, d = eng.lbg(10)
    C2, cnt = eng.update(A, 1 << 10)   # the single-step update goes through the exchange too
    np.savez(out, C=C, A=A, d=np.array([d]), C2=C2, cnt=cnt, info=np.array(eng.comm_info()))
    eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
