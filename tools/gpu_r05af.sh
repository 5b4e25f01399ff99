# Round 5 final record on the committed tree: the GPU suite, bench.py (default flags) + its kernel
# stats + PMC HBM passes (tools/gpu_bench.sh), C4 with the exact-sum rule (QVQ_KAHAN=0: no checks)
# for the floor, and the SQ counters of the C3 searches (tools/gpu_pmc_sq.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r05af
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r05af/gpu_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r05af/gpu_tests.log | tail -2
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_bench.sh r05af || exit $?
cd $R && QVQ_KAHAN=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline > gpurun_out/r05af/bench_exactsum.json 2> gpurun_out/r05af/bench_exactsum.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/r05af/bench_exactsum.json').read().strip().splitlines()[-1]); print('exact-sum rule: C3', d['ms_per_step'], 'C4', d['c4']['ms_per_step'])"
bash tools/gpu_pmc_sq.sh r05af_sq 4096,2,10 || exit $?
python3 tools/sq_view.py gpurun_out/r05af_sq 10 assign > gpurun_out/r05af/sq_search_levels.txt 2>&1 || true
echo record done
