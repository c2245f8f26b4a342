#!/bin/bash
# Round profile of the default bench (run on the GPU box): kernel-trace stats, then separate
# FETCH_SIZE / WRITE_SIZE passes for the HBM traffic of the dominant kernels.
#   bash tools/prof_bench.sh [tag]      -> gpurun_out/prof_<tag>/...
TAG=${1:-bench}
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
set -e
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o bench -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/prof_${TAG}_traffic -o $C -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_${TAG}_$C.log 2>&1
done
echo PROF_DONE
