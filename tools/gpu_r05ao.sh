# C3: pruning from K = 128 too (QVQ_U4_MAXK=64 QVQ_PRUNE_MINK=128) vs the default (from K = 256),
# interleaved three times, 20 steps, per-level search events
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ao
mkdir -p $O
cd $R
B="--steps 20 --warmup 3 --c4-steps 0 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline"
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py $B > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; return 1; }
  python3 -c "
import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); p=d['roofline']['per_level']
print('$n', 'C3', d['ms_per_step'], 'search us', [round(p[k]['avg_launch_ms']*1e3,1) for k in ['64','128','256','512']])"
}
for i in 1 2 3; do
run def_$i QVQ_X=0 && run p128_$i QVQ_U4_MAXK=64 QVQ_PRUNE_MINK=128 || exit 1
done
