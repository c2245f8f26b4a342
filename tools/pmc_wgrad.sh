#!/bin/bash
# usage: bash tools/pmc_wgrad.sh [experiment-lib-name ...]   (GPU box; summaries via tools/pmc_summary.py)
# PMC passes over the weight-gradient group launch (tools/kbench.py, 4M points): the in-tree build and xlibs/libpnr_<name>.so
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for N in head "$@"; do
  L=pointnerf-slam_amd/pnr/libpnr.so; [ "$N" != head ] && L=xlibs/libpnr_$N.so
  for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
    n=$(echo $C | cut -d' ' -f1)
    timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/pmcwg_$N -o $n -- python3 tools/kbench.py --precision f16x3 --reps 2 --lib $L > gpurun_out/pmcwg_${N}_$n.log 2>&1 || { echo FAIL $N $n; tail -5 gpurun_out/pmcwg_${N}_$n.log; exit 1; }
  done
  echo "== $N"; python3 tools/pmc_summary.py gpurun_out/pmcwg_$N k_wgrad16_group
done
