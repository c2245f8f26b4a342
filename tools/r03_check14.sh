#!/bin/bash
# round-3: probe zero-fill experiments (fill every row first / no fill: timing only)
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 150 python3 tools/gather_bench.py --reps 10 2>&1 | grep "k_gather " || exit 1
cp pointnerf-slam_amd/pnr/libpnr.so /tmp/libpnr_intree.so
for v in fillall nofill; do
  cp xlibs/libpnr_$v.so pointnerf-slam_amd/pnr/libpnr.so && echo $v && timeout -k 10 150 python3 tools/gather_bench.py --reps 10 2>&1 | grep "k_gather " || exit 1
done
