#!/bin/bash
# Two PMC passes over tools/gather_bench.py for the gather kernels.  Usage: bash tools/pmc_search.sh <tag>
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
T=${1:-cur}
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"; do
  n=$(echo $C | cut -d' ' -f1)
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/pmcs_$T -o $n -- python3 tools/gather_bench.py --reps 2 > gpurun_out/pmcs_${T}_$n.log 2>&1 || { echo FAIL $n; tail -5 gpurun_out/pmcs_${T}_$n.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmcs_$T gather_search
