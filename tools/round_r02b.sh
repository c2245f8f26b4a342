#!/bin/bash
# Round-2 profile + bench (GPU box): kernel-trace stats and PMC passes of the S-map / S-fwd bench
# (tools/prof_round.sh), FETCH_SIZE / WRITE_SIZE passes of the gather bench, then the default bench
# line.  bash tools/round_r02b.sh <tag>
set -e
TAG=$1
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
bash tools/prof_round.sh $TAG
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/prof_${TAG}_gtraffic -o $C -- \
    python3 tools/gather_bench.py --reps 2 > gpurun_out/prof_${TAG}_g$C.log 2>&1
  echo g$C
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_gather -o gb -- \
  python3 tools/gather_bench.py > gpurun_out/prof_${TAG}_gb.log 2>&1
echo gather-trace
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${TAG}.log 2>&1
tail -1 gpurun_out/bench_${TAG}.log | cut -c 1-300
echo ROUND_DONE
