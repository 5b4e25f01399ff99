set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
bash tools/gpu_kahan2.sh || exit 1
bash tools/gpu_c4trace.sh 2>&1 | tail -7
QVQ_CERT_TRACE=1 timeout -k 10 120 python3 tools/c3_bench_trace.py 2>&1 | tail -4
