# Round 5: the several-rank Kahan rule -- the new Kahan / communicator / rank tests first, then
# the whole GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05b
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kahan.py tests/test_gpu_multigpu.py -x -v --timeout 600 --timeout-method thread > $O/new_tests.log 2>&1; rc=$?
tail -30 $O/new_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -5 $O/gpu_tests.log
exit $rc
