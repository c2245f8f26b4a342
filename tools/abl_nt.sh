#!/bin/bash
# Streaming-store ablation (GPU box): gather_bench on the prebuilt variants in xlibs/
# (probe: NT zero fill only; ntc: + NT search c rows), then the full GPU suite on the probe build.
set -e
for r in 1 2; do for v in probe ntc; do
  cp xlibs/libpnr_$v.so pointnerf-slam_amd/pnr/libpnr.so
  echo "== $v"
  timeout -k 10 200 python3 tools/gather_bench.py --reps 20 2>&1 | grep "k_gather "
done; done
cp xlibs/libpnr_probe.so pointnerf-slam_amd/pnr/libpnr.so
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
