# Round-6 groundwork on the final tree: per-level kernel timelines of C3 and C4 (the last quantize
# of each trace, tools/level_view.py), the C4 host timeline, and the SQ counters of C4's searches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05aj
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in 4096,2,10 4096,4,12; do
  n=$(echo $c | tr , _)
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t_$n -o t -- python3 $R/tools/quick_timing.py $c > $O/t_$n.log 2>&1 || exit $?
  python3 $R/tools/level_view.py $O/t_$n/t_kernel_trace.csv --names > $O/levels_$n.txt 2>&1 || exit $?
done
cd $R && QVQ_HOST_TRACE=1 timeout -k 10 200 python3 tools/quick_timing.py 4096,4,12 > $O/c4_host.log 2>&1 || exit $?
bash tools/gpu_pmc_sq.sh r05aj_sq 4096,4,12 || exit $?
python3 tools/sq_view.py gpurun_out/r05aj_sq 12 wide > $O/sq_c4_wide_levels.txt 2>&1 || true
echo done
