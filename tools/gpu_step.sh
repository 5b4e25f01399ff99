# One iteration of the build -> measure loop: GPU parity + per-level trace (gpu_check.sh), a
# bench line without the CPU baseline, then A/B traces of the given ablations.
# usage: bash tools/gpu_step.sh ["name:VAR=val" ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_check.sh || exit $?
timeout -k 10 200 python $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_now.json 2> $R/gpurun_out/bench_now.err || exit $?
cut -c1-220 $R/gpurun_out/bench_now.json
if [ $# -gt 0 ]; then bash $R/tools/ab_env.sh 4096,2,10 "base:" "$@" || exit $?; fi
