# Kernel traces of one workload under several env settings (ablations; timing only).
# usage: bash tools/ab_env.sh CASE "name:VAR=val VAR2=val" ...   (name "base" = no vars)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
CASE=$1; shift
mkdir -p $R/gpurun_out/abe
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}; [ "$name" = "$spec" ] && vars=""
  timeout -k 10 180 env $vars rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/abe/$name -o t -- python3 $R/tools/quick_timing.py $CASE > $R/gpurun_out/abe/$name.log 2>&1 || { tail -5 $R/gpurun_out/abe/$name.log; exit 1; }
  echo "== $name ($vars)"; python3 $R/tools/trace_view.py $R/gpurun_out/abe/$name/t_kernel_trace.csv --compact
done
