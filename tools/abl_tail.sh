# Marginal cost of the per-level tail launches (QVQ_ABL_SKIP ablations, timing only):
# a C3 kernel trace per setting, with the per-quantize wall / busy span and the level table.
# usage: bash tools/abl_tail.sh [SKIP_MASKS...]   (default: 0 1 2 4 7)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/abl
cd /tmp && export TMPDIR=/tmp
for m in ${@:-0 1 2 4 7}; do
  QVQ_ABL_SKIP=$m timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/abl/m$m -o t -- python3 $R/tools/quick_timing.py 4096,2,10 > $R/gpurun_out/abl/m$m.log 2>&1 || exit 1
  echo "== QVQ_ABL_SKIP=$m"
  python3 $R/tools/gap_view.py $R/gpurun_out/abl/m$m/t_kernel_trace.csv | tail -2
  python3 $R/tools/trace_view.py $R/gpurun_out/abl/m$m/t_kernel_trace.csv --compact | tail -4
done
