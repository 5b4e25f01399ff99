# Small-K ring search (assign_small_ring_kernel, default) vs the 4-row groups (QVQ_SMALL_RING=0):
# the GPU suite, then C3 interleaved three times (20 steps each, per-level search events in the
# bench line), then a kernel trace of each for the per-level kernel times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ac
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/gpu_tests.log | tail -2
[ $rc -ne 0 ] && exit $rc
B="--steps 20 --warmup 3 --c4-steps 0 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline"
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py $B > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; return 1; }
  python3 -c "
import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); p=d['roofline']['per_level']
print('$n', 'C3', d['ms_per_step'], 'search us', [round(p[k]['avg_launch_ms']*1e3,1) for k in ['2','4','8','16','32']])"
}
for i in 1 2 3; do
run ring_$i QVQ_X=0 && run groups_$i QVQ_SMALL_RING=0 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  QVQ_SMALL_RING=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_ring$v -o t -- python3 $R/tools/quick_timing.py 4096,2,10 > $O/trace_ring$v.log 2>&1 || exit $?
  grep -h "small" $O/trace_ring$v/t_kernel_stats.csv | cut -d, -f1-4 | cut -c1-60,200- || true
done
