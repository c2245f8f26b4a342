#!/bin/bash
# Stall breakdown of the f16x3 eval forward, k_mlp_fwd16 (PNR_FWD_W16=0) against k_mlp_fwd16w (=1):
# one rocprofv3 --pmc pass per counter group on tools/kbench.py --eval-only, kernel trace only.
#   bash tools/pmc_w16.sh <tag> [lib]    -> gpurun_out/pmcw_<tag>_<w16>_<group>/, summary on stdout
TAG=${1:-r06}
LIB=${2:-pointnerf-slam_amd/pnr/libpnr.so}
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for W in 0 1; do
  i=0
  for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA"; do
    i=$((i+1))
    PNR_FWD_W16=$W timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/pmcw_${TAG}_${W}_$i -o k -- \
      python3 tools/kbench.py --precision f16x3 --reps 1 --points 2097152 --eval-only --lib $LIB > gpurun_out/pmcw_${TAG}_${W}_$i.log 2>&1 || { echo FAIL $W $i; tail -5 gpurun_out/pmcw_${TAG}_${W}_$i.log; exit 1; }
  done
  echo "== PNR_FWD_W16=$W"
  for i in 1 2; do python3 tools/pmc_summary.py gpurun_out/pmcw_${TAG}_${W}_$i k_mlp_fwd16; done
done
