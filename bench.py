"""bench.py -- LBG vector-quantization hot path on MI355X (BASELINE.json metric).

One step = one full LBGQuantizer::quantize (src/Quantizer.cpp:122-143): mean init plus
`bits` split levels, each one assign + one centroid update (+ the RCCL all-reduce of the
per-code-vector sums when N > 1), over a training set already resident in HBM.

Workload per rank: one 4096x4096 synthetic RGB image (seed 0x5EED+rank),
2x2 blocks (D = 12), 1024 code vectors -- BASELINE.json configs[2]/C3, the configuration
the reference CPU baseline (8.53 s) is quoted on.  N ranks train ONE joint codebook over
N images (weak scaling: per-GPU work fixed, one all-reduce per level).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

With --gpus N > 1 and no launcher environment (WORLD_SIZE unset), this script starts the N
rank processes itself (one per GPU, LOCAL_RANK = device index) before anything touches a GPU,
passes rank 0's JSON line through and exits with the worst rank status.  Under a launcher
WORLD_SIZE must equal --gpus.  --dry-run (CPU only): the ranks join the gloo control plane and
rank 0 prints what it would run, without touching a GPU.

Rank 0 prints one JSON line.  value = Mblocks/s = (blocks on all ranks) x levels x steps
/ max-over-ranks wall time / 1e6 (BASELINE.md section 2 definition).

Sub-objects of the same line (each timed the same way, barrier + synchronize around K steps,
max over ranks):
  c5   BASELINE.json config 5 -- the fixed 64-image 4096^2 batch, 2x2, K=1024, split over
       the N ranks (64/N images each) with the per-level RCCL all-reduce: STRONG scaling, the
       north-star 1->8 GPU curve.
  c4   (N = 1) config 4: 4096^2, 4x4 blocks (D=48), K=4096.
  end_to_end (N = 1) the drop-in's PCIe-inclusive compress: host raster -> H2D + tiling +
       quantize + the 16.8 MB index download (src/Compressor.cpp:118-123 timed region).
  cpu_baseline (N = 1) the oracle port, median of 5 at the box's cores and at 8 cores.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_F16_TFLOPS = 2500.0     # MI355X_MICROARCH.md: BF16/F16 MFMA ~2.5 PF dense (no sparsity)
PEAK_F32_VALU_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector peak (assign_small_kernel, K <= 32)
PEAK_HBM_GBS = 8000.0
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_hbm_latest.json")   # tools/pmc_summary.py output


def workload_key(args):
    return "%dx%d_b%d_bits%d_ipr%d" % (args.size, args.size, args.block, args.bits, args.images_per_rank)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--block", type=int, default=2)
    ap.add_argument("--bits", type=int, default=10)
    ap.add_argument("--images-per-rank", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, host cores)")
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--c5-images", type=int, default=64)
    ap.add_argument("--c5-steps", type=int, default=3, help="0 disables the c5 sub-object")
    ap.add_argument("--c4-steps", type=int, default=20, help="0 disables the c4 sub-object")
    ap.add_argument("--share-steps", type=int, default=3,
                    help="0 disables the c5_rank_share sub-object (N=8 per-rank share through a 1-rank RCCL communicator)")
    ap.add_argument("--e2e-reps", type=int, default=7, help="0 disables the end_to_end sub-object (the first rep after a reconfiguration is not timed; the second still pays first-use costs, hence the median of 7)")
    ap.add_argument("--exact-reps", type=int, default=2,
                    help="0 disables the exact_cie1931 sub-object (exact mode on the C3 raster's CIE1931 blocks)")
    ap.add_argument("--dry-run", action="store_true", help="CPU only: start the ranks, join gloo, print the plan")
    return ap.parse_args()


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """Start n rank processes of this script (RANK = LOCAL_RANK = r, WORLD_SIZE = n, rendezvous
    on 127.0.0.1) and wait for them.  The parent never touches a GPU, so the children start
    clean.  Rank 0's stdout (the JSON line) is the parent's; the other ranks' stdout goes to
    stderr.  If a rank fails, the others are stopped (they would wait at the next barrier)."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else sys.stderr))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0:
                rc = rc or code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


def dry_run(args, world, rank):
    """--dry-run: the ranks join the gloo control plane and agree on the shard plan; rank 0
    prints it.  No GPU is touched (tests/test_multirank_cpu.py runs this on the CPU box)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    n_img = args.c5_images
    share = [n_img // world + (1 if r < n_img % world else 0) for r in range(world)]
    t = torch.tensor([rank, os.getpid()], dtype=torch.int64)
    got = [torch.zeros_like(t) for _ in range(world)] if world > 1 else [t]
    if world > 1:
        dist.all_gather(got, t)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_joined": sorted(int(g[0]) for g in got),
                          "pids": [int(g[1]) for g in got], "c5_images_per_rank": share,
                          "headline": "one %dx%d image per rank, joint codebook" % (args.size, args.size)}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def _oracle_runs(args, threads, reps):
    cli = os.path.join(ROOT, "oracle", "build", "oracle_cli")
    if not os.path.exists(cli):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    out = subprocess.run([cli, "gen", str(args.size), str(0x5EED), str(args.block), str(args.block),
                          str(args.bits), str(threads), str(reps)], check=True, capture_output=True, text=True,
                         timeout=900).stdout
    return [json.loads(l) for l in out.strip().splitlines() if l.startswith("{")]


def cpu_baseline(args):
    """The oracle port (lbg_oracle.c, OpenMP on the same loops as the reference) on the
    same workload, on this host's cores: median of --cpu-reps full quantizes of one image at
    the box's core share (16 on the GPU box) and at 8 cores."""
    import statistics
    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    runs = {}
    for t in sorted({threads, min(8, threads)}, reverse=True):
        recs = _oracle_runs(args, t, args.cpu_reps)
        runs[t] = (statistics.median(r["quantize_s"] for r in recs), recs[0]["N"],
                   statistics.median(r["tile_s"] for r in recs))
    med, n, tile_s = runs[threads]
    mbps = n * args.bits / med / 1e6
    return {"value": round(mbps, 4), "unit": "Mblocks/s", "cores": threads, "kind": "port",
            "sample": "median of %d full quantizes (tiling excluded) of the rank-0 workload: %dx%d synthetic, %dx%d "
                      "blocks, %d levels, at %d threads: %.3f s (tiling %.3f s)%s"
                      % (args.cpu_reps, args.size, args.size, args.block, args.block, args.bits, threads, med, tile_s,
                         "".join("; at %d threads: %.3f s" % (t, v[0]) for t, v in runs.items() if t != threads)),
            "quantize_s_by_threads": {str(t): round(v[0], 4) for t, v in runs.items()}}


def synthetic_raster(S, seed):
    """SURVEY.md 8(d) generator in numpy (host raster for the PCIe-inclusive leg)."""
    with np.errstate(over="ignore"):
        p = np.arange(S * S, dtype=np.uint64)
        r, c = p // np.uint64(S), p % np.uint64(S)
        sm = [r * np.uint64(255) // np.uint64(S - 1), c * np.uint64(255) // np.uint64(S - 1),
              (r + c) * np.uint64(255) // np.uint64(2 * (S - 1))]
        out = np.empty((S * S, 3), np.uint8)
        for ch in range(3):
            z = (np.uint64(seed) << np.uint64(40)) ^ (p * np.uint64(3) + np.uint64(ch))
            z = z + np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            v = sm[ch].astype(np.int64) + (z % np.uint64(33)).astype(np.int64) - 16
            out[:, ch] = np.clip(v, 0, 255)
    return out.ravel()


def cie_blocks(rgb, S):
    """The 2x2 blocks (getBlocksAsVectorsFromImage: x-major blocks and pixels, src/Compressor.cpp:31-62)
    of an S x S raster's signed-char values, each pixel mapped through CIE1931 (src/ColorSpace.cpp:30-38):
    values off the byte grid, which only the exact mode (k_exact.hip) takes."""
    p = rgb.reshape(S * S, 3).view(np.int8).astype(np.float64)
    xyz = np.empty_like(p)
    xyz[:, 0] = (p[:, 0] * 0.490 + p[:, 1] * 0.310 + p[:, 2] * 0.200) / 0.17697
    xyz[:, 1] = (p[:, 0] * 0.17697 + p[:, 1] * 0.81240 + p[:, 2] * 0.01063) / 0.17697
    xyz[:, 2] = (p[:, 0] * 0 + p[:, 1] * 0.01 + p[:, 2] * 0.99) / 0.17697
    return np.ascontiguousarray(xyz.reshape(S // 2, 2, S // 2, 2, 3).transpose(0, 2, 1, 3, 4).reshape(-1, 12))


def exact_cie(args, eng, cpu):
    """Exact mode measured: qvq_lbg on the C3 raster's CIE1931 blocks (wall per quantize, inputs
    resident), and with cpu the oracle's Kahan rule on a bounded sample (512 x 512) beside it."""
    X = cie_blocks(synthetic_raster(args.size, 0x5EED), args.size)
    eng.set_vectors(X, exact=True)
    eng.lbg(args.bits, want_assign=False)   # warm-up (allocations)
    ms = []
    for _ in range(args.exact_reps):
        t = time.perf_counter()
        eng.lbg(args.bits, want_assign=False)
        ms.append((time.perf_counter() - t) * 1e3)
    tm = eng.timings()
    best = min(ms)
    out = {"workload": "C3 raster (%dx%d, 2x2 blocks) mapped through CIE1931, %d code vectors, exact mode "
                       "(fp64 search in nanoflann order + Kahan chains, the reference's arithmetic bit for bit)"
                       % (args.size, args.size, 1 << args.bits),
           "rows": int(X.shape[0]), "ms_per_quantize": round(best, 2), "reps": args.exact_reps,
           "Mblocks_per_s": round(X.shape[0] * args.bits / best / 1e3, 3),
           "assign_ms": [round(v, 2) for v in tm["assign_ms"]], "update_ms": [round(v, 2) for v in tm["update_ms"]],
           "phases": "per level, wall: assign = fp64 search + tie answers; update = stable sort + Kahan chains"}
    if cpu:
        from oracle import oracle
        s = 512
        Xs = cie_blocks(synthetic_raster(s, 0x5EED), s)
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        t = time.perf_counter()
        oracle.lbg(Xs, args.bits, sum_mode=0, threads=threads)
        cs = time.perf_counter() - t
        out["cpu_baseline"] = {"kind": "port", "sample": "%dx%d CIE1931 blocks (%d rows), %d levels, oracle Kahan rule"
                                                        % (s, s, Xs.shape[0], args.bits),
                               "cores": threads, "Mblocks_per_s": round(Xs.shape[0] * args.bits / cs / 1e6, 3)}
    del X
    return out


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))   # before anything touches a GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit("bench.py: WORLD_SIZE=%d but --gpus %d: launch one rank per GPU" % (world, args.gpus))
    if args.dry_run:
        return dry_run(args, world, rank)
    import torch
    import torch.distributed as dist
    import quant_amd

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)   # control plane only
    torch.cuda.set_device(local)

    def barrier():
        if world > 1:
            dist.barrier()

    eng = quant_amd.Engine(local)
    if world > 1:
        uid = [quant_amd.Engine.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init(world, rank, uid[0])   # RCCL over xGMI for the per-level sums
    comm_n, _, comm_kind = eng.comm_info()
    rccl_ranks = comm_n if comm_kind == quant_amd.COMM_RCCL else 0
    if world > 1 and rccl_ranks != world:
        sys.exit("bench.py: the engine joined %d RCCL ranks, expected %d" % (rccl_ranks, world))
    ipr = args.images_per_rank
    eng.set_synthetic(args.size, 0x5EED + rank * ipr, ipr, args.block, args.block, quant_amd.SCALED)
    n_local = eng.n
    D = eng.dim

    out = (np.empty((1 << args.bits, D), np.float64), np.zeros(1, np.float64))   # reused by every step
    for _ in range(args.warmup):
        eng.lbg(args.bits, want_assign=False, out=out)
    barrier()
    torch.cuda.synchronize()
    # The timed steps carry no instrumentation (an event record idles the GPU for a few us).
    eng.set_timing(-2)
    t0 = time.perf_counter()
    for step in range(args.steps):
        eng.lbg(args.bits, want_assign=False, out=out)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    # Then, outside the timed region, the same quantize again with HIP events around ONE
    # level's search launch per call (on the engine's stream), cycling through the levels:
    # the per-launch durations of the roofline below.
    launches, update_ms, flagged = [], [], []
    for step in range(max(args.steps, 2 * args.bits)):
        lvl = step % args.bits
        eng.set_timing(lvl)
        eng.lbg(args.bits, want_assign=False, out=out)
        a_ms, u_ms, f_rows = eng.level_timing(lvl)
        launches.append((1 << (lvl + 1), a_ms))
        update_ms.append(u_ms)
        flagged.append(f_rows)
    eng.set_timing(-2)
    tm_last = eng.timings()   # the last quantize's Kahan-rule statistics
    torch.cuda.synchronize()
    barrier()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
        n = torch.tensor([n_local], dtype=torch.int64)
        dist.all_reduce(n)
        n_total = int(n[0])
    else:
        n_total = n_local

    levels = args.bits
    value = n_total * levels * args.steps / elapsed / 1e6
    ms_per_step = elapsed * 1e3 / args.steps

    # Roofline of the dominant kernel, the search (assign_mf32_kernel: v_mfma_f32_32x32x16_f16
    # for K >= 64, assign_small_kernel: expanded fp32 scores for K <= 32; centroid sums fused),
    # from HIP events around the launches on the engine's stream.  Algorithmic work per launch
    # = 3*K_l*D flop per block x blocks.
    flops = sum(3.0 * K * D * n_local for K, _ in launches)
    secs = sum(ms for _, ms in launches) * 1e-3
    achieved = flops / secs / 1e12
    avg_launch_s = secs / len(launches)
    # per level (K): the largest K is the dominant launch of a quantize.  Each level's search is
    # priced against the peak of the unit it runs on: K <= 32 expanded fp32 scores on the VALU
    # (assign_small_kernel), K >= 64 f16 MFMA tiles (assign_mf32_kernel); and against HBM with its
    # algorithmic bytes (Dp bytes of codes in, a 4-byte index out per block)
    Dp = (D + 3) & ~3
    assign_bytes = n_local * (Dp + 4)
    pmc = None
    try:
        pmc = json.load(open(PMC_SUMMARY))
        if pmc.get("workload") != workload_key(args):
            pmc = None
    except (OSError, ValueError, KeyError):
        pmc = None

    def pmc_kernel(K):
        """PMC HBM bytes per launch of level K's search kernel (tools/pmc_summary.py names)."""
        if not pmc:
            return None
        if K <= 32:
            name = "assign_small_kernel<%d,fused>" % K
        elif K <= 128:
            name = "assign_mf32_kernel<fused,staged,U4,tag>"
        elif K <= 512:
            name = "assign_mf32_kernel<fused,staged,U8,tag,prune>"
        else:
            name = "assign_mf32_kernel<fused,global,U8,tag,prune>"
        v = pmc["kernels"].get(name)
        return v["hbm_bytes"] if v else None

    by_k = {}
    for K, ms in launches:
        by_k.setdefault(K, []).append(ms)
    per_level = {}
    for K, v in sorted(by_k.items()):
        t = sum(v) / len(v) * 1e-3
        tf = 3.0 * K * D * n_local / t / 1e12
        valu = K <= 32
        peak = PEAK_F32_VALU_TFLOPS if valu else PEAK_F16_TFLOPS
        gbs = assign_bytes / t / 1e9
        per_level[str(K)] = {"avg_launch_ms": round(t * 1e3, 5), "TFLOPs": round(tf, 2),
                             "unit_peak": "fp32 VALU %.1f TF" % peak if valu else "f16 MFMA dense %.0f TF" % peak,
                             "frac": round(tf / peak, 4),
                             "hbm_GBps": round(gbs, 1), "hbm_frac": round(gbs / PEAK_HBM_GBS, 4),
                             "traffic": pmc_kernel(K)}
    Kdom = max(by_k)
    dom = per_level[str(Kdom)]
    traffic = dom["traffic"]
    traffic_src = os.path.relpath(PMC_SUMMARY, ROOT) if traffic is not None else None
    # the mean (once per quantize, HBM-bound: Dp bytes per block) with events around it alone
    mean_ms = []
    eng.set_timing(-3)
    for _ in range(5):
        eng.lbg(args.bits, want_assign=False, out=out)
        mean_ms.append(eng.timings()["mean_ms"])
    eng.set_timing(-2)
    mean_t = sum(mean_ms) / len(mean_ms) * 1e-3
    mean_gbs = n_local * Dp / mean_t / 1e9
    upd_secs = sum(update_ms) * 1e-3
    upd_bytes = len(update_ms) * n_local * (((D + 3) & ~3) + 4)
    result = {
        "metric": "Mblocks/s (assign+update)",
        "value": round(value, 3),
        "unit": "Mblocks/s",
        "n_gpus": world,
        "rccl_ranks": rccl_ranks,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f16 MFMA search on exact integer byte operands + fp64 recheck, exact integer centroid sums",
        "data": "synthetic (SURVEY.md 8(d) generator, seed 0x5EED+image), resident in HBM",
        "config": {"workload": "C3: %dx%d synthetic RGB per image, %dx%d blocks (D=%d), %d code vectors, "
                               "%d image(s) per rank, joint codebook" % (args.size, args.size, args.block,
                                                                         args.block, D, 1 << args.bits, ipr),
                   "blocks_per_rank": n_local, "levels": levels, "parallelism": "dp%d" % world},
        "lbg_iters_per_s": round(levels * args.steps / elapsed, 3),
        # the dominant kernel: the largest level's search (K = 1024 at C3), one launch per quantize
        "roofline": {"bound": "mfma", "kernel": "qvq::assign_mf32_kernel (v_mfma_f32_32x32x16_f16, pruned, fused "
                                                 "exact sums), the K=%d level's search" % Kdom,
                     "achieved": dom["TFLOPs"], "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
                     "frac": dom["frac"], "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes": assign_bytes, "avg_launch_ms": dom["avg_launch_ms"],
                     "flop_per_block": "3*K*D", "flop_per_launch": 3 * Kdom * D * n_local,
                     "timing": "HIP events around one level's search per quantize, levels in rotation, in quantizes "
                               "after the timed steps",
                     "per_level": per_level,
                     # every level's search launches together (the mix a quantize runs)
                     "all_levels": {"achieved": round(achieved, 3), "frac_of_f16_peak": round(achieved / PEAK_F16_TFLOPS, 4),
                                    "avg_launch_ms": round(avg_launch_s * 1e3, 5), "launches": len(launches)},
                     "mean_kernel": {"avg_launch_ms": round(mean_t * 1e3, 5), "algorithmic_bytes": n_local * Dp,
                                     "hbm_GBps": round(mean_gbs, 1), "hbm_frac": round(mean_gbs / PEAK_HBM_GBS, 4)},
                     "hbm_peak_GBps": PEAK_HBM_GBS},
        "update_kernel": ({"avg_launch_ms": round(upd_secs * 1e3 / max(1, len(update_ms)), 5),
                           "achieved_GBps": round(upd_bytes / upd_secs / 1e9, 1), "peak_GBps": PEAK_HBM_GBS}
                          if upd_secs else "fused into the search (LDS u64 atomics of exact integer terms)"),
        "flagged_rows_per_step": flagged[-1],
        # the indices' rule: the reference's (Kahan centroid bits decide the tie rows, on every
        # rank count) unless QVQ_KAHAN=0 selects the exact-sum rule (A/B)
        "index_rule": "exact-sum" if os.environ.get("QVQ_KAHAN") == "0" else "kahan (reference)",
        "kahan_checks": {"redo": tm_last["kahan_redo"], "cross_rank_cell_sums": tm_last["kahan_relays"],
                         "tie_export_overflow": tm_last["tie_overflow"]},
    }
    def timed(fn, steps, warmup):
        """Max-over-ranks wall of `steps` calls of fn after `warmup`, barrier + sync on both sides."""
        for _ in range(warmup):
            fn()
        barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        barrier()
        el = time.perf_counter() - t
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt[0])
        return el

    # C5: the fixed 64-image batch split over the ranks, one joint codebook (strong scaling)
    if args.c5_steps > 0:
        n_img = args.c5_images
        share = [n_img // world + (1 if r < n_img % world else 0) for r in range(world)]
        start = sum(share[:rank])
        eng.set_synthetic(args.size, 0x5EED + start, share[rank], 2, 2, quant_amd.SCALED)
        eng.set_timing(-2)
        out5 = (np.empty((1 << args.bits, eng.dim), np.float64), np.zeros(1, np.float64))
        el = timed(lambda: eng.lbg(args.bits, want_assign=False, out=out5), args.c5_steps, 1)
        n5 = n_img * ((args.size + 1) // 2) ** 2
        result["c5"] = {"workload": "C5: %d x %dx%d synthetic (seeds 0x5EED..+%d), 2x2 blocks, %d code vectors, "
                                    "one joint codebook, %d image(s) on this rank" % (n_img, args.size, args.size,
                                                                                       n_img - 1, 1 << args.bits,
                                                                                       share[rank]),
                        "value": round(n5 * args.bits * args.c5_steps / el / 1e6, 3), "unit": "Mblocks/s",
                        "ms_per_step": round(el * 1e3 / args.c5_steps, 3), "steps": args.c5_steps, "warmup": 1,
                        "n_gpus": world, "scaling": "strong", "blocks_total": n5,
                        "images_per_rank": share, "collective": "RCCL all-reduce per level" if world > 1 else "none"}
    if world == 1 and args.c4_steps > 0:
        eng.set_synthetic(args.size, 0x5EED, 1, 4, 4, quant_amd.SCALED)
        eng.set_timing(-2)
        out4 = (np.empty((1 << 12, eng.dim), np.float64), np.zeros(1, np.float64))
        # (3 warmups: the first C4 call sizes the context's and the trees' pooled buffers)
        el = timed(lambda: eng.lbg(12, want_assign=False, out=out4), args.c4_steps, 3)
        result["c4"] = {"workload": "C4: %dx%d synthetic, 4x4 blocks (D=48), 4096 code vectors" % (args.size, args.size),
                        "value": round(eng.n * 12 * args.c4_steps / el / 1e6, 3), "unit": "Mblocks/s",
                        "ms_per_step": round(el * 1e3 / args.c4_steps, 3), "steps": args.c4_steps, "warmup": 3}
    if world == 1 and args.share_steps > 0:
        # one rank's share of C5 at N=8, under the communicator schedule (a 1-rank RCCL
        # communicator: the all-reduce per level, kd ties and reduce as with N ranks) and under
        # the one-rank schedule: the per-rank workload of the 8-GPU run, not a scaling curve
        n_share = max(1, args.c5_images // 8)
        share_res = {}
        for label, with_comm in (("one_rank_schedule", False), ("rccl_schedule", True)):
            e2 = quant_amd.Engine(local)
            try:
                if with_comm:
                    e2.comm_init(1, 0, quant_amd.Engine.comm_unique_id())
                e2.set_synthetic(args.size, 0x5EED, n_share, 2, 2, quant_amd.SCALED)
                e2.set_timing(-2)
                o2 = (np.empty((1 << args.bits, e2.dim), np.float64), np.zeros(1, np.float64))
                el = timed(lambda: e2.lbg(args.bits, want_assign=False, out=o2), args.share_steps, 1)
                kind = e2.comm_info()[2]
                share_res[label] = {"ms_per_step": round(el * 1e3 / args.share_steps, 3),
                                    "Mblocks_per_s": round(e2.n * args.bits * args.share_steps / el / 1e6, 3),
                                    "communicator": "RCCL, 1 rank" if kind == quant_amd.COMM_RCCL else "none"}
            finally:
                e2.close()
        r1, rc = share_res["one_rank_schedule"]["ms_per_step"], share_res["rccl_schedule"]["ms_per_step"]
        result["c5_rank_share"] = {"workload": "the N=8 per-rank share of C5: %d x %dx%d synthetic images, 2x2 blocks, "
                                               "%d code vectors on one GPU (per-rank workload, not a scaling curve)"
                                               % (n_share, args.size, args.size, 1 << args.bits),
                                   "steps": args.share_steps, "warmup": 1, **share_res,
                                   "rccl_over_one_rank": round(rc / r1, 4)}
    if world == 1 and args.e2e_reps > 0:
        # the drop-in's compress region from a host raster: H2D + tiling + quantize + indices D2H
        rgb = synthetic_raster(args.size, 0x5EED)
        Cb = np.empty((1 << args.bits, 3 * args.block * args.block), np.float64)
        times = []
        for r in range(args.e2e_reps + 1):
            t = time.perf_counter()
            eng.set_images(rgb, 1, args.size, args.size, args.block, args.block, quant_amd.SCALED)
            _, A_host, _ = eng.lbg(args.bits, out=(Cb, np.zeros(1, np.float64)))
            if r:
                times.append(time.perf_counter() - t)
        times.sort()
        med = times[len(times) // 2]
        result["end_to_end"] = {"what": "host raster -> qvq_set_images (50 MB H2D + tiling) + qvq_lbg + %d-byte "
                                        "index download; not the headline" % (A_host.size * 4),
                                "ms": round(med * 1e3, 3), "Mblocks_per_s": round(n_local * args.bits / med / 1e6, 3),
                                "reps": args.e2e_reps}
        result["end_to_end_ms"] = round(med * 1e3, 3)
    if world == 1 and args.exact_reps > 0:
        e3 = quant_amd.Engine(local)
        try:
            result["exact_cie1931"] = exact_cie(args, e3, not args.no_cpu_baseline)
        finally:
            e3.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cb = cpu_baseline(args)
            result["cpu_baseline"] = cb
            result["speedup_vs_cpu"] = round(value / cb["value"], 1)
        except Exception as e:   # the GPU number stands on its own
            result["cpu_baseline"] = {"error": str(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
