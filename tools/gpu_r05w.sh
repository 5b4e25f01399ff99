# host timelines (QVQ_HOST_TRACE) of C4 quantizes: the reference's rule and the exact-sum rule
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05w
mkdir -p $O
cd $R
QVQ_HOST_TRACE=1 timeout -k 10 120 python3 tools/quick_timing.py 4096,4,12 > $O/kahan.log 2>&1 || exit $?
QVQ_KAHAN=0 QVQ_HOST_TRACE=1 timeout -k 10 120 python3 tools/quick_timing.py 4096,4,12 > $O/exact.log 2>&1 || exit $?
QVQ_HOST_TRACE=1 timeout -k 10 120 python3 tools/quick_timing.py 4096,2,10 > $O/c3.log 2>&1 || exit $?
grep -c "host trace" $O/kahan.log
