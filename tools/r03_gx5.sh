#!/bin/bash
# Gather at HEAD: search PMC passes (issue / wait mix), FETCH_SIZE / WRITE_SIZE passes, kernel-trace stats
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/pmc_search.sh r03h > gpurun_out/pmcs_r03h_summary.txt 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/prof_r03h_gtraffic -o $C -- \
    python3 tools/gather_bench.py --reps 2 > gpurun_out/prof_r03h_g$C.log 2>&1
  echo g$C
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03h_gather -o gb -- \
  python3 tools/gather_bench.py > gpurun_out/prof_r03h_gb.log 2>&1
echo GX5_DONE
