set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05e
mkdir -p $O
cd $R
QVQ_KAHAN_DEBUG=1 timeout -k 10 120 python3 tools/comm_diag.py > $O/diag.log 2>&1; rc=$?
grep -v "^qvq kahan: K [0-9]* ties [0-9]* ([0-9]* distinct) verified" $O/diag.log | tail -40
exit $rc
