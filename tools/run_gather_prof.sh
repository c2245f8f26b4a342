cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 tools/gather_bench.py > gpurun_out/gb1.log 2>&1 && cat gpurun_out/gb1.log && timeout -k 10 900 bash tools/pmc_gather.sh > gpurun_out/pmcg.log 2>&1 && python3 tools/pmc_summary.py gpurun_out/pmcg gather > gpurun_out/pmcg_summary.txt && cat gpurun_out/pmcg_summary.txt
