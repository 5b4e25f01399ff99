# suite + C3/C4 bench (short searches replay before their near sets) + traces
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05q
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('C3', d['ms_per_step'], 'C4', d['c4']['ms_per_step'], d['kahan_checks'])"
QVQ_CERT_TRACE=1 timeout -k 10 120 python3 tools/quick_timing.py 4096,2,10 4096,4,12 > $O/cert_trace.log 2>&1 || exit $?
grep "K 1024 \|K 4096 \|K 2048 " $O/cert_trace.log | tail -6
QVQ_CERT_EARLY=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline > $O/bench_noearly.json 2> $O/bench_noearly.err || { tail -5 $O/bench_noearly.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$O/bench_noearly.json').read().strip().splitlines()[-1]); print('noearly C3', d['ms_per_step'], 'C4', d['c4']['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
QVQ_CERT_TRACE=1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/tr_c4 -o t -- python3 $R/tools/quick_timing.py 4096,4,12 > $O/tr_c4.log 2>&1 || exit $?
QVQ_CERT_TRACE=1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/tr_c3 -o t -- python3 $R/tools/quick_timing.py 4096,2,10 > $O/tr_c3.log 2>&1 || exit $?
cd $R
python3 tools/tail_view.py $(ls $O/tr_c4/*/t_kernel_trace.csv $O/tr_c4/t_kernel_trace.csv 2>/dev/null | head -1) 2 > $O/tail_c4.txt || true
python3 tools/tail_view.py $(ls $O/tr_c3/*/t_kernel_trace.csv $O/tr_c3/t_kernel_trace.csv 2>/dev/null | head -1) 1 > $O/tail_c3.txt || true
tail -n 4 $O/tail_c4.txt; tail -n 4 $O/tail_c3.txt
