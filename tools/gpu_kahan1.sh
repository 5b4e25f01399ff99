# Reference-rule (Kahan) parity corpus, then the whole GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_kahan.py -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/kahan1.log 2>&1 || { tail -30 $R/gpurun_out/kahan1.log; exit 1; }
tail -3 $R/gpurun_out/kahan1.log
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -v --timeout 120 --timeout-method thread > $R/gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E 'passed|failed' $R/gpurun_out/pytest_gpu.log | tail -3
grep -E 'FAILED' $R/gpurun_out/pytest_gpu.log | head -30
exit $rc
