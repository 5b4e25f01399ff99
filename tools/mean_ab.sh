# mean_sums_kernel time by grid cap (QVQ_MEAN_GRID), C3, kernel stats per setting.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/meanab; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for g in 128 256 512 1024; do
  QVQ_MEAN_GRID=$g timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g$g -o t -- python3 $R/tools/quick_timing.py 4096,2,10 > $O/g$g.log 2>&1 || exit $?
  echo "grid $g: $(grep -h mean_sums $O/g$g/t_kernel_stats.csv | cut -d, -f2-5)"
done
