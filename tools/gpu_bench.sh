# Official-style measurement on one MI355X: bench.py, kernel-trace stats of the same
# command, and FETCH_SIZE / WRITE_SIZE passes (separate, counters only) -> profiles/.
# usage: bash tools/gpu_bench.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py "$@" > $R/gpurun_out/$TAG/bench.json 2> $R/gpurun_out/$TAG/bench.err || exit $?
cat $R/gpurun_out/$TAG/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace -o b -- python3 $R/bench.py --no-cpu-baseline "$@" > $R/gpurun_out/$TAG/trace.log 2>&1 || exit $?
# counter passes on the headline (C3) workload only: no c5 / c4 / end_to_end sub-runs
C3ONLY="--c5-steps 0 --c4-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/$TAG/fetch -o f -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 $C3ONLY "$@" > $R/gpurun_out/$TAG/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/$TAG/write -o w -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 $C3ONLY "$@" > $R/gpurun_out/$TAG/write.log 2>&1 || exit $?
cd $R && python3 tools/pmc_summary.py $R/gpurun_out/$TAG/pmc_hbm.json $R/gpurun_out/$TAG/fetch $R/gpurun_out/$TAG/write 4096x4096_b2_bits10_ipr1 > /dev/null || exit $?
echo done
