# GPU parity suite, per-level timings and a kernel trace of one C3 quantize.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/quick_timing.py 512,2,10 4096,2,10 4096,4,12 > gpurun_out/quick.log 2>&1 && cat gpurun_out/quick.log && bash tools/gpu_prof.sh
