# One parametrised runner for every GPU call (replaces the per-call gpu_r0*.sh scripts).
# usage (on the box, from the repo root):  bash tools/gpu.sh TAG STEP [STEP ...]
# Each STEP runs under its own time limit; the first failing step ends the call.  Output goes to
# gpurun_out/TAG/.  Steps:
#   suite               pytest -m gpu (log: gpu_tests.log)
#   suite:EXPR          only the tests matching -k EXPR
#   record              bench.py defaults + kernel stats of the same command + FETCH/WRITE PMC passes
#   bench[:ARGS]        bench.py with ARGS (commas for spaces), JSON to bench_N.json
#   ab:N:SPEC;SPEC...   N interleaved C3 runs per SPEC "name=VAR=v,VAR2=v" (20 steps, per-level events)
#   timeline:CASE       kernel trace of tools/quick_timing.py CASE (e.g. 4096,4,12), no timing events -> levels_CASE.txt
#   host:CASE           QVQ_HOST_TRACE=1 host timeline of CASE -> host_CASE.log
#   sq:CASE:KIND        SQ counters of CASE's searches (tools/gpu_pmc_sq.sh)
#   py:SCRIPT[:ARGS]    python3 SCRIPT ARGS (commas for spaces), log to py_N.log
#   callab:N            N ABBA pairs of tools/c4_calls.py (40 C4 calls each) with lib_base and lib -> callab.txt
#   libab:N             N interleaved bench runs (C3 20 steps, C4 10) of quant_amd/lib_base/libqvq.so
#                       (the build before a change) and quant_amd/lib, in ABBA order -> base_I.json / new_I.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  echo "== step $n: $step"
  case $kind in
  suite)
    K=(); [ -n "$arg" ] && K=(-k "$arg")
    (cd $R && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread "${K[@]}" > $O/gpu_tests.log 2>&1)
    rc=$?; grep -E "passed|failed|error" $O/gpu_tests.log | tail -3; [ $rc -ne 0 ] && exit $rc ;;
  record)
    (cd /tmp && bash $R/tools/gpu_bench.sh $TAG) || exit $? ;;
  bench)
    A=${arg//,/ }
    (cd $R && timeout -k 10 400 python3 bench.py $A > $O/bench_$n.json 2> $O/bench_$n.err) || { tail -5 $O/bench_$n.err; exit 1; }
    tail -c 600 $O/bench_$n.json ;;
  ab)
    reps=${arg%%:*}; specs=${arg#*:}
    B="--steps 20 --warmup 3 --c4-steps 0 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline"
    for i in $(seq 1 $reps); do
      IFS=';' read -ra SP <<< "$specs"
      for s in "${SP[@]}"; do
        name=${s%%=*}; vars=${s#*=}; [ "$name" = "$s" ] && vars="QVQ_NONE=0"
        (cd $R && env ${vars//,/ } timeout -k 10 300 python3 bench.py $B > $O/${name}_$i.json 2> $O/${name}_$i.err) || { tail -3 $O/${name}_$i.err; exit 1; }
        python3 -c "
import json; d=json.loads(open('$O/${name}_$i.json').read().strip().splitlines()[-1]); p=d['roofline']['per_level']
print('${name}_$i', 'C3', d['ms_per_step'], 'search us', {k: round(p[k]['avg_launch_ms']*1e3,1) for k in sorted(p, key=int)})"
      done
    done ;;
  timeline)
    c=${arg//,/_}
    (cd /tmp && QT_EVENTS=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t_$c -o t -- python3 $R/tools/quick_timing.py $arg > $O/t_$c.log 2>&1) || exit $?
    (cd $R && python3 tools/level_view.py $O/t_$c/t_kernel_trace.csv --names > $O/levels_$c.txt 2>&1) || exit $?
    tail -25 $O/levels_$c.txt ;;
  host)
    c=${arg//,/_}
    (cd $R && QVQ_HOST_TRACE=1 timeout -k 10 200 python3 tools/quick_timing.py $arg > $O/host_$c.log 2>&1) || exit $?
    tail -5 $O/host_$c.log ;;
  sq)
    c=${arg%%:*}; k=${arg#*:}
    (cd $R && bash tools/gpu_pmc_sq.sh ${TAG}_sq $c) || exit $?
    (cd $R && python3 tools/sq_view.py gpurun_out/${TAG}_sq 12 $k > $O/sq_$k.txt 2>&1) || true ;;
  py)
    s=${arg%%:*}; a=${arg#*:}; [ "$a" = "$arg" ] && a=""
    (cd $R && timeout -k 10 400 python3 -u $s ${a//,/ } > $O/py_$n.log 2>&1) || { tail -20 $O/py_$n.log; exit 1; }
    tail -20 $O/py_$n.log ;;
  callab)
    for i in $(seq 1 ${arg:-3}); do
      for k in $( [ $((i % 2)) = 1 ] && echo "base new new base" || echo "new base base new" ); do
        L=""; [ $k = base ] && L=$R/quant_amd/lib_base/libqvq.so
        echo -n "$k " >> $O/callab.txt
        (cd $R && QVQ_LIB=$L timeout -k 10 200 python3 tools/c4_calls.py 4096,4,12 40 >> $O/callab.txt 2> $O/callab.err) || { tail -5 $O/callab.err; exit 1; }
      done
    done
    cat $O/callab.txt ;;
  libab)
    B="--steps 20 --warmup 3 --c4-steps 10 --c5-steps 0 --e2e-reps 0 --share-steps 0 --exact-reps 0 --no-cpu-baseline"
    for i in $(seq 1 ${arg:-4}); do   # (order alternating, ABBA: a drift over the call cancels)
      for k in $( [ $((i % 2)) = 1 ] && echo "base new" || echo "new base" ); do
        L=""; [ $k = base ] && L=$R/quant_amd/lib_base/libqvq.so
        (cd $R && QVQ_LIB=$L timeout -k 10 300 python3 bench.py $B > $O/${k}_$i.json 2> $O/${k}_$i.err) || { tail -5 $O/${k}_$i.err; exit 1; }
      done
    done
    (cd $R && python3 -c "
import json, sys
for k in ('base', 'new'):
    r = [json.load(open('$O/%s_%d.json' % (k, i))) for i in range(1, ${arg:-4} + 1)]
    print(k, 'C3 ms', ' / '.join('%.4f' % x['ms_per_step'] for x in r), '| C4 ms', ' / '.join('%.3f' % x['c4']['ms_per_step'] for x in r))
" | tee $O/libab.txt) ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps done"
