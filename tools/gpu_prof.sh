# Kernel trace of one C3 quantize (per-kernel timeline for tools/trace_view.py).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof3 -o t -- python3 $GRAFT_REPO_ROOT/tools/quick_timing.py ${1:-4096,2,10} > $GRAFT_REPO_ROOT/gpurun_out/prof3.log 2>&1
rc=$?; tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof3.log; exit $rc
