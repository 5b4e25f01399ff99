# SQ instruction / stall counters of the search kernel on one workload (separate passes,
# counters only).  usage: bash tools/gpu_pmc_sq.sh TAG "S,bw,bits"
set -o pipefail
TAG=$1; CASE=${2:-4096,2,10}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_SMEM" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS_ATOMIC SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $P --kernel-include-regex "${REGEX:-assign}" --output-format csv -d $R/gpurun_out/$TAG/p$i -o p -- python3 $R/tools/quick_timing.py $CASE > $R/gpurun_out/$TAG/p$i.log 2>&1 || exit $?
done
echo done
