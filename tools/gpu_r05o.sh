# the Kahan test file three times after double-buffering the published codebook
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05o
mkdir -p $O
cd $R
for i in 1 2 3; do
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kahan.py -q --timeout 200 --timeout-method thread > $O/k$i.log 2>&1; echo "run $i rc $?"; tail -n 1 $O/k$i.log; grep FAILED $O/k$i.log
done
exit 0
