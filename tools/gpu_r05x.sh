# suite; C3/C4 bench; host timeline of C4 (the checks' set-up over the helper threads)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05x
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -n 2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
B="--steps 20 --warmup 5 --c4-steps 20 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline"
for i in 1 2; do
timeout -k 10 300 python3 bench.py $B > $O/bench$i.json 2> $O/bench$i.err || { tail -5 $O/bench$i.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench$i.json').read().strip().splitlines()[-1]); print('C3', d['ms_per_step'], 'C4', d['c4']['ms_per_step'])"
done
QVQ_HOST_TRACE=1 timeout -k 10 120 python3 tools/quick_timing.py 4096,4,12 > $O/c4_host.log 2>&1 || exit $?
python3 - <<'PY'
t=open('gpurun_out/r05x/c4_host.log').read().split('qvq host trace:')[-1].split('\n{')[0]
for l in t.strip().splitlines():
    if any(x in l for x in ('K2048','K4096','results','joined','return')): print(l)
PY
