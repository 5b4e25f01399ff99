# Round 5 final record: the GPU suite, bench.py (default flags) + its kernel stats + PMC HBM passes
# (tools/gpu_bench.sh), and C4 with the exact-sum rule (QVQ_KAHAN=0: no checks) for the floor
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r05aa
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r05aa/gpu_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r05aa/gpu_tests.log | tail -2
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_bench.sh r05aa || exit $?
cd $R && QVQ_KAHAN=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline > gpurun_out/r05aa/bench_exactsum.json 2> gpurun_out/r05aa/bench_exactsum.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/r05aa/bench_exactsum.json').read().strip().splitlines()[-1]); print('exact-sum rule: C3', d['ms_per_step'], 'C4', d['c4']['ms_per_step'])"
