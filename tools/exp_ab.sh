#!/bin/bash
# A/B kernel timing of experiment builds + rocprof kernel stats of the in-tree build (GPU box)
#   bash tools/exp_ab.sh <tag> <lib...>
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp
cd $R
for L in "$@"; do
  echo "== $L"
  timeout -k 10 150 python3 tools/kbench.py --precision f16x3 --reps 5 --lib $L
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o kb -- \
  python3 tools/kbench.py --precision f16x3 --reps 3 > gpurun_out/prof_${TAG}_kb.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_g -o gb -- \
  python3 tools/gather_bench.py > gpurun_out/prof_${TAG}_gb.log 2>&1
tail -3 gpurun_out/prof_${TAG}_gb.log
echo EXP_DONE
