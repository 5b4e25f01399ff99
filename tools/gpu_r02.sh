# Round-2 GPU check: parity suite, bench (all sub-objects), kernel trace of the bench.
# usage: bash tools/gpu_r02.sh TAG
set -o pipefail
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o t -- python3 $R/bench.py --no-cpu-baseline --e2e-reps 1 > $O/prof.log 2>&1
rc=$?; tail -2 $O/prof.log; exit $rc
