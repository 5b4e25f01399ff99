"""N > 1 path on CPU (gloo, world_size 2): rows sharded across ranks, per-rank exact
partial sums in the engine's exchange format [hi K*D][lo K*D][cnt K] (u64), one
all-reduce, the engine's finaliser -> must equal the single-process centroids bit for bit
(the property that makes 1/2/4/8-GPU runs produce identical codebooks)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from oracle import oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import quant_amd
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, codes = oracle.tile(oracle.gen_image(128), 128, 128, 2, 2)
    K = 32
    A = (np.arange(len(X)) * 2654435761 % K).astype(np.uint32)
    lo_r, hi_r = rank * len(X) // world, (rank + 1) * len(X) // world
    hi, lo = quant_amd.host_row_terms(codes[lo_r:hi_r])
    H = np.zeros((K, 12), np.uint64)
    L = np.zeros((K, 12), np.uint64)
    np.add.at(H, A[lo_r:hi_r], hi)
    np.add.at(L, A[lo_r:hi_r], lo)
    cnt = np.bincount(A[lo_r:hi_r], minlength=K).astype(np.uint64)
    buf = torch.from_numpy(np.concatenate([H.ravel(), L.ravel(), cnt]).astype(np.int64))
    dist.all_reduce(buf)
    s = buf.numpy().astype(np.uint64)
    C = quant_amd.host_finalize(s[:K * 12].reshape(K, 12), s[K * 12:2 * K * 12].reshape(K, 12), s[2 * K * 12:])
    q.put((rank, C))
    dist.destroy_process_group()


def test_sharded_sums_equal_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    X, _ = oracle.tile(oracle.gen_image(128), 128, 128, 2, 2)
    A = (np.arange(len(X)) * 2654435761 % 32).astype(np.uint32)
    ref = oracle.centroids(X, A, 32, sum_mode=1)
    for r in range(world):
        np.testing.assert_array_equal(res[r], ref)


def test_bench_launches_ranks_dry_run():
    """bench.py --gpus N without a launcher starts N rank processes that join the gloo control
    plane (the driver's `python bench.py --gpus N` form); --dry-run keeps them off the GPU."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    for n in (2, 3):
        out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(n), "--dry-run"],
                             capture_output=True, text=True, timeout=300, env=env, cwd=root)
        assert out.returncode == 0, out.stderr[-2000:]
        line = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
        assert line["n_gpus"] == n and line["ranks_joined"] == list(range(n))
        assert len(set(line["pids"])) == n and sum(line["c5_images_per_rank"]) == 64


def test_bench_refuses_mismatched_world():
    """Under a launcher, WORLD_SIZE must equal --gpus (a mis-launched run must not look valid)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                         capture_output=True, text=True, timeout=120, env=env, cwd=root)
    assert out.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in out.stderr
