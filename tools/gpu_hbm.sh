# HBM-bound kernels: mean sums (inside a C3 quantize) and the decode gather, kernel trace + stats.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-hbm}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/q -o t -- python3 $R/tools/quick_timing.py 4096,2,10 > $O/q.log 2>&1 || exit $?
cd $R && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d -o t -- python3 $R/tools/decode_bench.py > $O/d.log 2>&1 || exit $?
grep -h "mean_sums\|decode" $O/q/t_kernel_stats.csv $O/d/t_kernel_stats.csv | cut -c1-200
