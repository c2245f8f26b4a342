#!/bin/bash
# round-3: gather search ablations (experiment builds swapped in; timing only)
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 150 python3 tools/gather_bench.py --reps 5 2>&1 | grep "k_gather " || exit 1
for v in nonet nofeat; do
  cp xlibs/libpnr_$v.so pointnerf-slam_amd/pnr/libpnr.so && echo $v && timeout -k 10 150 python3 tools/gather_bench.py --reps 5 2>&1 | grep "k_gather " || exit 1
done
