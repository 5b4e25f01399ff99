# Kernel traces of one workload for several libqvq builds (timing only, no parity).
# usage: bash tools/ab_trace.sh CASE DIR1 DIR2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
CASE=$1; shift
mkdir -p $R/gpurun_out/abt
cd /tmp && export TMPDIR=/tmp
for d in "$@"; do
  export QVQ_LIB=$R/quant_amd/$d/libqvq.so
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/abt/$d -o t -- python3 $R/tools/quick_timing.py $CASE > $R/gpurun_out/abt/$d.log 2>&1 || exit 1
  echo "== $d"; python3 $R/tools/trace_view.py $R/gpurun_out/abt/$d/t_kernel_trace.csv --last-quantize --compact
done
