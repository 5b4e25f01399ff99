# the Kahan test file with the per-level timing events on (the old default) and off
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05l
mkdir -p $O
cd $R
QVQ_TIMING=-1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kahan.py -q --timeout 200 --timeout-method thread > $O/kahan_timing.log 2>&1; echo "timing rc $?"; tail -n 4 $O/kahan_timing.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kahan.py -q --timeout 200 --timeout-method thread > $O/kahan_default.log 2>&1; echo "default rc $?"; tail -n 4 $O/kahan_default.log
