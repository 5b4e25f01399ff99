# The Kahan centroid evaluator against the oracle, then the Kahan-rule corpus, then a C3 trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
QVQ_KAHAN_DEBUG=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_kahan.py -x -v --timeout 200 --timeout-method thread > gpurun_out/kahan2.log 2>&1 || { tail -40 gpurun_out/kahan2.log; exit 1; }
grep -E "passed|failed|qvq kahan" gpurun_out/kahan2.log | tail -30
