# The whole reference-bit split through the step-by-step chains (QVQ_KAHAN_DIRECT_MAX=1e9: every
# cell's chain in ks_direct_kernel instead of the segment functions, whose build took ~2.3 ms of
# the ~3.3 ms whole split at C4, profiles/r05ag): C4 interleaved, default vs full+direct vs direct
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ah
mkdir -p $O
cd $R
B="--steps 3 --warmup 1 --c4-steps 20 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline"
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py $B > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', 'C3', d['ms_per_step'], 'C4', d['c4']['ms_per_step'], 'redo', d['kahan_checks'])"
}
for i in 1 2; do
run def_$i QVQ_X=0 && run fulldirect_$i QVQ_FULL_SPLIT=1 QVQ_KAHAN_DIRECT_MAX=1000000000 && run direct_$i QVQ_KAHAN_DIRECT_MAX=1000000000 || exit 1
done
cd /tmp && export TMPDIR=/tmp
QVQ_FULL_SPLIT=1 QVQ_KAHAN_DIRECT_MAX=1000000000 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fd -o t -- python3 $R/tools/quick_timing.py 4096,4,12 > $O/fd.log 2>&1 || exit $?
grep -h "ks_" $O/fd/t_kernel_stats.csv | cut -c1-60,200-400 || true
