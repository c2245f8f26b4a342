#!/bin/bash
# round-3: gather search variants (early rejection in-tree; two-sample feature rounds)
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 150 python3 tools/gather_bench.py --reps 10 2>&1 | grep "k_gather " || exit 1
cp pointnerf-slam_amd/pnr/libpnr.so /tmp/libpnr_intree.so
for v in feat2 feat2w6; do
  cp xlibs/libpnr_$v.so pointnerf-slam_amd/pnr/libpnr.so && echo $v && timeout -k 10 150 python3 tools/gather_bench.py --reps 10 2>&1 | grep "k_gather " || exit 1
done
cp /tmp/libpnr_intree.so pointnerf-slam_amd/pnr/libpnr.so && echo intree-again && timeout -k 10 150 python3 tools/gather_bench.py --reps 10 2>&1 | grep "k_gather "
