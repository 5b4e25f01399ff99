# exact mode after the loader fix: parity tests, C3 CIE1931 timing, A/B of the chain kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r04g
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_exact.py > gpurun_out/r04g/exact_tests.log 2>&1 || { tail -20 gpurun_out/r04g/exact_tests.log; exit 1; }
tail -2 gpurun_out/r04g/exact_tests.log
timeout -k 10 240 python3 tools/exact_c3.py --check-side 256 > gpurun_out/r04g/exact_c3.log 2>&1 || { tail -5 gpurun_out/r04g/exact_c3.log; exit 1; }
cat gpurun_out/r04g/exact_c3.log
QVQ_EXACT_LDS_MAXK=64 timeout -k 10 240 python3 tools/exact_c3.py > gpurun_out/r04g/exact_c3_maxk64.log 2>&1 || { tail -5 gpurun_out/r04g/exact_c3_maxk64.log; exit 1; }
cat gpurun_out/r04g/exact_c3_maxk64.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04g/trace -o x -- python3 $R/tools/exact_c3.py --reps 1 > $R/gpurun_out/r04g/trace.log 2>&1 || { tail -5 $R/gpurun_out/r04g/trace.log; exit 1; }
head -12 $R/gpurun_out/r04g/trace/x_kernel_stats.csv | cut -c1-200
