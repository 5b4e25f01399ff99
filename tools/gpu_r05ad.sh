# Certificate aggregates: leaves with their running values in registers and their rows prefetched
# (default) vs one row at a time (QVQ_AGG_ROWS=1); C4 interleaved three times, 20 steps each, after
# the GPU suite; then one C4 host timeline of the default
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ad
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/gpu_tests.log | tail -2
[ $rc -ne 0 ] && exit $rc
B="--steps 3 --warmup 1 --c4-steps 20 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline"
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py $B > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', 'C3', d['ms_per_step'], 'C4', d['c4']['ms_per_step'])"
}
for i in 1 2 3; do
run regs_$i QVQ_X=0 && run rows_$i QVQ_AGG_ROWS=1 || exit 1
done
QVQ_HOST_TRACE=1 timeout -k 10 300 python3 bench.py $B > $O/trace.json 2> $O/trace_host.log || exit 1
