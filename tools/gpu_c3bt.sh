# Kernel trace of bench-style C3 quantizes (all streams).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/c3bt -o t -- python3 $R/tools/c3_bench_trace.py > $R/gpurun_out/c3bt.log 2>&1 || { tail -20 $R/gpurun_out/c3bt.log; exit 1; }
grep -E "quantize|redo" $R/gpurun_out/c3bt.log
QVQ_CERT_TRACE=1 timeout -k 10 120 python3 $R/tools/c3_bench_trace.py 2>&1 | tail -12
