# Kernel trace of C4 quantizes with the whole reference-bit split on (QVQ_FULL_SPLIT=1): where the
# ~2.7 ms of the device's whole split go (ks_* kernels), for tools/level_view.py-style reading
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
QVQ_FULL_SPLIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/full -o t -- python3 $R/tools/quick_timing.py 4096,4,12 > $O/full.log 2>&1 || exit $?
grep -h "ks_\|kahan" $O/full/t_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120 || true
