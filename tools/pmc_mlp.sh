cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_COUNT"; do
  n=$(echo $C | cut -d' ' -f1)
  timeout -k 10 200 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_${PREC:-f16x3} -o $n -- python3 tools/kbench.py --points 2097152 --reps 2 --precision ${PREC:-f16x3} > gpurun_out/pmc_$n.log 2>&1 || { echo FAIL $n; tail -5 gpurun_out/pmc_$n.log; exit 1; }
done
echo DONE
