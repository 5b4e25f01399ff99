# the Kahan test file alone on one box: default, then with the certificate preparation off
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05k
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kahan.py -x -q --timeout 200 --timeout-method thread > $O/kahan_default.log 2>&1; echo "default rc $?"; tail -n 3 $O/kahan_default.log
QVQ_CERT_PREP=0 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kahan.py -x -q --timeout 200 --timeout-method thread > $O/kahan_noprep.log 2>&1; echo "noprep rc $?"; tail -n 3 $O/kahan_noprep.log
