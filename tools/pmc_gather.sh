#!/bin/bash
# PMC passes for the point-gather kernels (one rocprofv3 --pmc pass per counter group, kernel
# trace only), on tools/gather_bench.py.  Usage (on the GPU box): bash tools/pmc_gather.sh [args]
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
ARGS="$@"
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INST_CYCLES_VMEM" \
         "TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  n=$(echo $C | cut -d' ' -f1)
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/pmcg -o $n -- python3 tools/gather_bench.py --reps 2 $ARGS > gpurun_out/pmcg_$n.log 2>&1 || { echo FAIL $n; tail -5 gpurun_out/pmcg_$n.log; exit 1; }
done
echo DONE
