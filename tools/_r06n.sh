#!/bin/bash
# after the contraction fix of map_row_point: bitwise A/B (fused map rows vs k_map_pts), full GPU tests + smoke
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
L=pointnerf-slam_amd/pnr/libpnr.so
PNR_MAP_ROWS_FUSE=0 timeout -k 10 200 python3 tools/lib_ab.py --lib $L --out /tmp/a.pt > gpurun_out/r06n_bit.log 2>&1 || { echo "lib_ab a failed"; tail -20 gpurun_out/r06n_bit.log; exit 1; }
timeout -k 10 200 python3 tools/lib_ab.py --lib $L --out /tmp/b.pt --ref /tmp/a.pt >> gpurun_out/r06n_bit.log 2>&1 || { echo "lib_ab b failed"; tail -20 gpurun_out/r06n_bit.log; exit 1; }
grep -c "bitwise True" gpurun_out/r06n_bit.log
bash tools/gpu_round.sh tests
