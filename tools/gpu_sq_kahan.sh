# SQ counters of the Kahan kernels (k_kahan.hip) over C3 quantizes (separate passes, counters only).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/sqk
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $P --kernel-include-regex "ks_" --output-format csv -d $R/gpurun_out/sqk/p$i -o p -- python3 $R/tools/quick_timing.py 4096,2,10 > $R/gpurun_out/sqk/p$i.log 2>&1 || exit $?
done
python3 $R/tools/sq_view.py $R/gpurun_out/sqk 10 ks_
