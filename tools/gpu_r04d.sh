# C3-only kernel stats (gpurun_out/r04c) then the C4 certificate trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_r04c.sh || exit $?
echo
cd $R
QVQ_CERT_TRACE=1 timeout -k 10 120 python3 tools/c4_trace.py > gpurun_out/c4t.log 2>&1 || exit $?
tail -14 gpurun_out/c4t.log
