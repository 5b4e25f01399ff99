# C3-only kernel stats of bench.py (the headline workload alone) -> gpurun_out/r04c.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r04c
cd /tmp && export TMPDIR=/tmp
C3ONLY="--c5-steps 0 --c4-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04c/trace -o b -- python3 $R/bench.py --steps 20 --warmup 3 $C3ONLY > $R/gpurun_out/r04c/trace.log 2>&1 || exit $?
grep '^{' $R/gpurun_out/r04c/trace.log | head -c 400
