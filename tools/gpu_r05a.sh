# Round 5 first call: the GPU suite on the starting tree, then the unfused-sum A/B on C3
# (QVQ_FUSE=0: search without LDS sums + a separate sums pass) with kernel traces and SQ counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05a
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
cd /tmp && export TMPDIR=/tmp
for spec in "base:" "nofuse:QVQ_FUSE=0"; do
  name=${spec%%:*}; vars=${spec#*:}
  timeout -k 10 180 env $vars rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o t -- python3 $R/tools/quick_timing.py 4096,2,10 > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 1; }
  echo "== $name"; python3 $R/tools/trace_view.py $O/$name/t_kernel_trace.csv --compact | tail -40
done
for spec in "base:" "nofuse:QVQ_FUSE=0"; do
  name=${spec%%:*}; vars=${spec#*:}
  i=0
  for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_SMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS_ATOMIC SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU"; do
    i=$((i+1))
    timeout -s KILL 90 env $vars rocprofv3 --pmc $P --kernel-include-regex "assign|update|sorted|reduce" --output-format csv -d $O/sq_$name/p$i -o p -- python3 $R/tools/quick_timing.py 4096,2,10 > $O/sq_${name}_p$i.log 2>&1 || { tail -5 $O/sq_${name}_p$i.log; exit 1; }
  done
done
echo done
