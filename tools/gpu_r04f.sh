# Round 4 final record: the GPU suite, then bench.py + its kernel stats + PMC HBM passes (tools/gpu_bench.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/gpu_bench.sh r04f --steps 20 --warmup 3
