# decode kernel time by grid cap (QVQ_DECODE_GRID), C3 size.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/decab; mkdir -p $O
cd $R
for g in 512 1024 2048 4096; do
  QVQ_DECODE_GRID=$g timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g$g -o t -- python3 $R/tools/decode_bench.py > $O/g$g.log 2>&1 || exit $?
  echo "grid $g: $(grep -h decode_rows $O/g$g/t_kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f1-4)"
done
