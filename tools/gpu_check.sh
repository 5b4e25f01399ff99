# GPU parity suite then a compact kernel trace of one C3 quantize (the usual loop step).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E 'passed|failed|error' $R/gpurun_out/pytest_gpu.log | tail -3
[ $rc -ne 0 ] && { grep -E 'FAILED|Error|assert' $R/gpurun_out/pytest_gpu.log | head -20; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/chk -o t -- python3 $R/tools/quick_timing.py ${1:-4096,2,10} > $R/gpurun_out/chk.log 2>&1 || exit $?
python3 $R/tools/trace_view.py $R/gpurun_out/chk/t_kernel_trace.csv --compact
