set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
QVQ_CERT_TRACE=1 timeout -k 10 120 python3 tools/c4_trace.py > gpurun_out/c4t.log 2>&1
tail -14 gpurun_out/c4t.log
QVQ_SPECULATE=0 timeout -k 10 120 python3 tools/c4_trace.py 2>&1 | tail -3
