# exact mode: parity tests, then C3 CIE1931 timing with the LDS chains and the per-thread chains (A/B)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_exact.py > gpurun_out/exact_tests.log 2>&1 || { tail -20 gpurun_out/exact_tests.log; exit 1; }
tail -2 gpurun_out/exact_tests.log
timeout -k 10 240 python3 tools/exact_c3.py --check-side 256 > gpurun_out/exact_c3.log 2>&1 || { tail -5 gpurun_out/exact_c3.log; exit 1; }
cat gpurun_out/exact_c3.log
QVQ_EXACT_CHAINS=thread timeout -k 10 400 python3 tools/exact_c3.py --reps 1 > gpurun_out/exact_c3_thread.log 2>&1 || { tail -5 gpurun_out/exact_c3_thread.log; exit 1; }
cat gpurun_out/exact_c3_thread.log
echo
bash tools/gpu_r04d.sh
echo "== A/B check stream priority"
for p in 1 0; do
QVQ_VSTREAM_PRIO=$p timeout -k 10 120 python3 tools/c4_trace.py > gpurun_out/c4t_p$p.log 2>&1 || exit 1
echo "prio=$p c4: $(grep -h 'quantize' gpurun_out/c4t_p$p.log | tr '\n' ' ')"
QVQ_VSTREAM_PRIO=$p timeout -k 10 120 python3 tools/quick_timing.py 4096,2,10 > gpurun_out/c3q_p$p.log 2>&1 || exit 1
echo "prio=$p c3: $(grep -o '"wall_ms": [0-9.]*' gpurun_out/c3q_p$p.log | tr '\n' ' ')"
done
