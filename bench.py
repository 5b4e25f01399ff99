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

Rank 0 prints one JSON line.  value = Mblocks/s = (blocks on all ranks) x levels x steps
/ max-over-ranks wall time / 1e6 (BASELINE.md section 2 definition).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_F16_TFLOPS = 2500.0     # MI355X_MICROARCH.md: BF16/F16 MFMA ~2.5 PF dense (no sparsity)
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
    return ap.parse_args()


def cpu_baseline(args):
    """The oracle port (lbg_oracle.c, OpenMP on the same loops as the reference) on the
    same workload, on this host's cores: one full quantize of one image."""
    from oracle import oracle  # noqa: F401  (builds liboracle if missing)
    cli = os.path.join(ROOT, "oracle", "build", "oracle_cli")
    if not os.path.exists(cli):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    out = subprocess.run([cli, "gen", str(args.size), str(0x5EED), str(args.block), str(args.block),
                          str(args.bits), str(threads), "1"], check=True, capture_output=True, text=True,
                         timeout=600).stdout
    rec = json.loads(out.strip().splitlines()[-1])
    n = rec["N"]
    mbps = n * args.bits / rec["quantize_s"] / 1e6
    return {"value": round(mbps, 4), "unit": "Mblocks/s", "cores": threads, "kind": "port",
            "sample": "one full quantize (tiling excluded) of the rank-0 workload: %dx%d synthetic, %dx%d "
                      "blocks, %d levels; quantize %.3f s, tiling %.3f s"
                      % (args.size, args.size, args.block, args.block, args.bits, rec["quantize_s"],
                         rec["tile_s"])}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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
    ipr = args.images_per_rank
    eng.set_synthetic(args.size, 0x5EED + rank * ipr, ipr, args.block, args.block, quant_amd.SCALED)
    n_local = eng.n
    D = eng.dim

    import numpy as np
    out = (np.empty((1 << args.bits, D), np.float64), np.zeros(1, np.float64))   # reused by every step
    for _ in range(args.warmup):
        eng.lbg(args.bits, want_assign=False, out=out)
    barrier()
    torch.cuda.synchronize()
    # Each step times ONE level's search launch with HIP events on the engine's stream,
    # cycling through the levels (an event record idles the GPU for a few us, so timing
    # every level would tax the measured step).
    launches, update_ms, flagged = [], [], []
    t0 = time.perf_counter()
    for step in range(args.steps):
        lvl = step % args.bits
        eng.set_timing(lvl)
        eng.lbg(args.bits, want_assign=False, out=out)
        a_ms, u_ms, f_rows = eng.level_timing(lvl)
        launches.append((1 << (lvl + 1), a_ms))
        update_ms.append(u_ms)
        flagged.append(f_rows)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
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

    # Roofline of the dominant kernel, the search (assign_mfma_kernel: f16 MFMA 16x16x32 for
    # K >= 64, assign_small_kernel: direct fp32 for K <= 32; centroid sums fused), from HIP
    # events around the launches on the engine's stream.  Algorithmic work per launch =
    # 3*K_l*D flop per block x blocks.
    flops = sum(3.0 * K * D * n_local for K, _ in launches)
    secs = sum(ms for _, ms in launches) * 1e-3
    achieved = flops / secs / 1e12
    avg_launch_s = secs / len(launches)
    # its HBM view: codes in (Dp bytes per block) + index out (4 bytes per block)
    assign_bytes = n_local * (((D + 3) & ~3) + 4)
    traffic, traffic_src = None, None
    try:
        pmc = json.load(open(PMC_SUMMARY))
        ks = [v for k, v in pmc["kernels"].items() if k.startswith("assign_")]
        if ks and pmc.get("workload") == workload_key(args):
            tot = sum(v["hbm_bytes"] * v["launches"] for v in ks)
            traffic = round(tot / sum(v["launches"] for v in ks))
            traffic_src = os.path.relpath(PMC_SUMMARY, ROOT)
    except (OSError, ValueError, KeyError):
        pass
    upd_secs = sum(update_ms) * 1e-3
    upd_bytes = len(update_ms) * n_local * (((D + 3) & ~3) + 4)
    result = {
        "metric": "Mblocks/s (assign+update)",
        "value": round(value, 3),
        "unit": "Mblocks/s",
        "n_gpus": world,
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
        "roofline": {"bound": "mfma", "kernel": "search: qvq::assign_mfma_kernel (v_mfma_f32_16x16x32_f16, K >= 64) / "
                                                 "qvq::assign_small_kernel (direct fp32, K <= 32), fused sums",
                     "achieved": round(achieved, 3), "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / PEAK_F16_TFLOPS, 4), "traffic": traffic,
                     "traffic_source": traffic_src, "avg_launch_ms": round(avg_launch_s * 1e3, 5),
                     "launches": len(launches), "flop_per_block": "3*K*D",
                     "timing": "HIP events around one level's search per step, levels in rotation",
                     "hbm_view": {"algorithmic_bytes_per_launch": assign_bytes,
                                  "achieved_GBps": round(assign_bytes / avg_launch_s / 1e9, 1),
                                  "peak_GBps": PEAK_HBM_GBS}},
        "update_kernel": ({"avg_launch_ms": round(upd_secs * 1e3 / max(1, len(update_ms)), 5),
                           "achieved_GBps": round(upd_bytes / upd_secs / 1e9, 1), "peak_GBps": PEAK_HBM_GBS}
                          if upd_secs else "fused into the search (LDS u64 atomics of exact integer terms)"),
        "flagged_rows_per_step": flagged[-1],
    }
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
