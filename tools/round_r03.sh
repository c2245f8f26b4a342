#!/bin/bash
# Round-3 profile (GPU box): kernel-trace stats and PMC passes of the S-map / S-fwd bench
# (tools/prof_round.sh), FETCH_SIZE / WRITE_SIZE passes and the kernel trace of the gather bench.
#   bash tools/round_r03.sh <tag>   (the bench line itself runs in a call of its own)
set -e
TAG=$1
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/prof_round.sh $TAG
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/prof_${TAG}_gtraffic -o $C -- \
    python3 tools/gather_bench.py --reps 2 > gpurun_out/prof_${TAG}_g$C.log 2>&1
  echo g$C
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_gather -o gb -- \
  python3 tools/gather_bench.py > gpurun_out/prof_${TAG}_gb.log 2>&1
echo gather-trace
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_f1000 -o f -- \
  python3 bench.py --rays 1000 --graph --steps 50 --warmup 3 --no-extras --no-cpu-baseline --no-gather \
  > gpurun_out/prof_${TAG}_f1000.log 2>&1
echo ROUND_PROF_DONE
