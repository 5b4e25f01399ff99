# the Kahan test file three times with the per-level timing events on and three times off
# (an intermittent "second quantize differs" seen in r05i / r05k)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05m
mkdir -p $O
cd $R
for i in 1 2 3; do
QVQ_TIMING=-1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kahan.py -q --timeout 200 --timeout-method thread > $O/t$i.log 2>&1; echo "timing $i rc $?"; tail -n 1 $O/t$i.log; grep FAILED $O/t$i.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kahan.py -q --timeout 200 --timeout-method thread > $O/d$i.log 2>&1; echo "default $i rc $?"; tail -n 1 $O/d$i.log; grep FAILED $O/d$i.log
done
exit 0
