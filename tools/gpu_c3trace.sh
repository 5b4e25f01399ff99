# Kernel trace of C3 quantizes (quick_timing) with the per-level timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c3t -o t -- python3 $R/tools/quick_timing.py ${1:-4096,2,10} > $R/gpurun_out/c3t.log 2>&1 || { tail -20 $R/gpurun_out/c3t.log; exit 1; }
cat $R/gpurun_out/c3t.log | grep '^{'
python3 $R/tools/trace_view.py $R/gpurun_out/c3t/t_kernel_trace.csv --compact 2>&1 | tail -60
