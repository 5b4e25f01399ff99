# C4 A/B, interleaved three times, 20 steps each: checks on one thread while a tree builds (default) or not
# exact-sum rule (no checks) -- the run-to-run spread on one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05z
mkdir -p $O
cd $R
B="--steps 3 --warmup 1 --c4-steps 20 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline"
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py $B > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', 'C4', d['c4']['ms_per_step'])"
}
for i in 1 2 3; do
run yield_$i QVQ_X=0 && run noyield_$i QVQ_CHECK_YIELD=0 || exit 1
done
