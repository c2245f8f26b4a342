#!/bin/bash
# k_map_pts fused into the training forward (kMapRows): bitwise A/B against PNR_MAP_ROWS_FUSE=0, room0 timing, full GPU tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
L=pointnerf-slam_amd/pnr/libpnr.so
PNR_MAP_ROWS_FUSE=0 timeout -k 10 200 python3 tools/lib_ab.py --lib $L --out /tmp/a.pt > gpurun_out/r06m_bit.log 2>&1 || { echo "lib_ab a failed"; tail -20 gpurun_out/r06m_bit.log; exit 1; }
timeout -k 10 200 python3 tools/lib_ab.py --lib $L --out /tmp/b.pt --ref /tmp/a.pt >> gpurun_out/r06m_bit.log 2>&1 || { echo "lib_ab b failed"; tail -20 gpurun_out/r06m_bit.log; exit 1; }
grep bitwise gpurun_out/r06m_bit.log
O=gpurun_out/r06m_ab.log; : > $O
for r in 1 2 3; do for F in 1 0; do
  PNR_MAP_ROWS_FUSE=$F timeout -k 10 200 python3 bench.py --workload room0 --steps 200 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/r06m_$F.json 2>gpurun_out/r06m_err.log || { echo "bench failed"; tail -5 gpurun_out/r06m_err.log; exit 1; }
  echo "$r fuse=$F $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06m_$F.json | head -1)" >> $O
done; done
cat $O
bash tools/gpu_round.sh tests
