# Pruning from K = 256 with 8-code-vector units there (the new default) vs the unpruned 4-unit
# search at K = 256 (QVQ_U4_MAXK=256 QVQ_PRUNE_MINK=512): the GPU suite on the new default, then C3
# interleaved three times (20 steps, per-level search events)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05am
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
print('$n', 'C3', d['ms_per_step'], 'search us', [round(p[k]['avg_launch_ms']*1e3,1) for k in ['128','256','512','1024']])"
}
for i in 1 2 3; do
run p256_$i QVQ_X=0 && run p512_$i QVQ_U4_MAXK=256 QVQ_PRUNE_MINK=512 || exit 1
done
