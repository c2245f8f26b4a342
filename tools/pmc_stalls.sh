#!/bin/bash
# Stall breakdown of the split MLP kernels (GPU box): one rocprofv3 --pmc pass per counter group on
# tools/kbench.py (f16x3), kernel trace only.  SQ_WAIT_ANY (parked at s_waitcnt / barrier) +
# SQ_WAIT_INST_ANY (issue stall) + SQ_ACTIVE_INST_ANY ~ SQ_WAVE_CYCLES (MI355X_MICROARCH.md).
#   bash tools/pmc_stalls.sh <tag>   -> gpurun_out/pmcs_<tag>_<group>/
TAG=${1:-r02}
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/pmcs_${TAG}_$i -o k -- \
    python3 tools/kbench.py --precision f16x3 --reps 1 --points 2097152 > gpurun_out/pmcs_${TAG}_$i.log 2>&1 || { echo FAIL $i; tail -5 gpurun_out/pmcs_${TAG}_$i.log; exit 1; }
  echo pass $i
done
echo PMCS_DONE
