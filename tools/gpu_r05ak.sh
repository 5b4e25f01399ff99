# C4's small levels: the wide MFMA search from K = 32 / 64 (QVQ_WIDE_MIN_K) vs the VALU search below
# K = 128 (default): C4 interleaved twice (20 steps), a per-level trace of each, and the D=48 GPU
# tests under the lower threshold
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ak
mkdir -p $O
cd $R
B="--steps 3 --warmup 1 --c4-steps 20 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline"
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py $B > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', 'C4', d['c4']['ms_per_step'])"
}
for i in 1 2; do
run def_$i QVQ_X=0 && run w64_$i QVQ_WIDE_MIN_K=64 && run w32_$i QVQ_WIDE_MIN_K=32 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for m in 128 64 32; do
  QVQ_WIDE_MIN_K=$m timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t$m -o t -- python3 $R/tools/quick_timing.py 4096,4,12 > $O/t$m.log 2>&1 || exit $?
  python3 $R/tools/level_view.py $O/t$m/t_kernel_trace.csv > $O/levels_$m.txt 2>&1 || exit $?
  head -8 $O/levels_$m.txt
done
cd $R && QVQ_WIDE_MIN_K=32 timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "wide or 4x4 or c4 or C4 or 48 or exact" > $O/tests_w32.log 2>&1; rc=$?
tail -2 $O/tests_w32.log
exit $rc
