# the Kahan test file twice with each of three builds (QVQ_LIB): round start, the first commit of
# this session, the current tree -- which change brought the intermittent second-quantize mismatch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05n
mkdir -p $O
cd $R
for lib in ab/libqvq_4afe3ec.so ab/libqvq_31d2c6b.so libqvq.so; do
for i in 1 2; do
n=$(basename $lib .so)_$i
QVQ_LIB=$R/quant_amd/lib/$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kahan.py -q --timeout 200 --timeout-method thread > $O/$n.log 2>&1; echo "$n rc $?"; tail -n 1 $O/$n.log; grep FAILED $O/$n.log
done
done
exit 0
