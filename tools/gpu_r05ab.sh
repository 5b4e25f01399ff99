# The whole-split 48-D check (QVQ_FULL_SPLIT, default on) against the certificate's cells
# (QVQ_FULL_SPLIT=0): GPU suite on the default, then C4 interleaved three times, 20 steps each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ab
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
run full_$i QVQ_X=0 && run cells_$i QVQ_FULL_SPLIT=0 || exit 1
done
QVQ_HOST_TRACE=1 timeout -k 10 300 python3 bench.py $B > $O/trace_full.json 2> $O/trace_full.err || exit 1
