# Kahan-rule GPU tests, then the certificate's phases on bench-style C3 quantizes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
bash tools/gpu_kahan2.sh || exit 1
QVQ_CERT_TRACE=1 timeout -k 10 120 python3 tools/c3_bench_trace.py > gpurun_out/ct.log 2>&1
tail -8 gpurun_out/ct.log
