# Round 5: the Kahan / communicator / rank tests, the whole GPU suite, then the checks' phases
# (QVQ_CERT_TRACE) on C3 and C4 and the whole-level Kahan cost (rocprof).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05d
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kahan.py tests/test_gpu_multigpu.py -x -v --timeout 600 --timeout-method thread > $O/new_tests.log 2>&1; rc=$?
tail -30 $O/new_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
QVQ_CERT_TRACE=1 timeout -k 10 120 python3 tools/quick_timing.py 4096,2,10 4096,4,12 > $O/cert_trace.log 2>&1 || exit $?
grep -c "qvq kahan" $O/cert_trace.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kcost -o k -- python3 $R/tools/kahan_cost.py > $O/kcost.log 2>&1 || exit $?
cat $O/kcost.log
echo done
