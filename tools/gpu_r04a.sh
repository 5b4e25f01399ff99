# Round 4: Kahan tests, a C3 kernel trace (Kahan on), then the GPU suite and one bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu_kahan2.sh || exit 1
bash tools/gpu_c3trace.sh || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
grep FAILED gpurun_out/pytest_gpu.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/bench_r04a.json 2> gpurun_out/bench_r04a.err; tail -c 3000 gpurun_out/bench_r04a.json
