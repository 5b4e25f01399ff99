# C3: K = 256 (now pruned, 8-code-vector units) with the wave run reduction into one LDS sums copy
# (QVQ_SUM_COPIES_MAXK=128) vs the default per-lane atomics into several copies; interleaved three
# times, then the GPU suite under the candidate setting
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ap
mkdir -p $O
cd $R
B="--steps 20 --warmup 3 --c4-steps 0 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline"
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py $B > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; return 1; }
  python3 -c "
import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); p=d['roofline']['per_level']
print('$n', 'C3', d['ms_per_step'], 'search us', [round(p[k]['avg_launch_ms']*1e3,1) for k in ['128','256','512']])"
}
for i in 1 2 3; do
run def_$i QVQ_X=0 && run runs256_$i QVQ_SUM_COPIES_MAXK=128 || exit 1
done
QVQ_SUM_COPIES_MAXK=128 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_runs256.log 2>&1; rc=$?
tail -1 $O/gpu_tests_runs256.log
exit $rc
