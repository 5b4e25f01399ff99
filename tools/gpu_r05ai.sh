# Fused sums into several LDS copies (K = 64..512): adjacent rows at the same index added in
# registers first (default) vs every row's own atomics (QVQ_PAIR_SUMS=0): the GPU suite, then C3
# interleaved three times (20 steps, per-level search events), then the LDS conflict counters
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ai
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
print('$n', 'C3', d['ms_per_step'], 'search us', [round(p[k]['avg_launch_ms']*1e3,1) for k in ['64','128','256','512','1024']])"
}
for i in 1 2 3; do
run pair_$i QVQ_X=0 && run row_$i QVQ_PAIR_SUMS=0 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  QVQ_PAIR_SUMS=$v timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS_ATOMIC SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS --kernel-include-regex assign --output-format csv -d $O/sq$v -o p -- python3 $R/tools/quick_timing.py 4096,2,10 > $O/sq$v.log 2>&1 || exit $?
done
echo done
