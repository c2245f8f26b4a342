#!/bin/bash
# round-3 experiment: persistent feature-branch forward (spills) vs the per-tile launch, map-points
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 bench.py --workload map-points --steps 3 --warmup 1 --no-cpu-baseline --no-gather > gpurun_out/mp17a.log 2>&1 || exit 1
echo "intree $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mp17a.log | head -1)"
cp pointnerf-slam_amd/pnr/libpnr.so /tmp/libpnr_intree.so
cp xlibs/libpnr_pst.so pointnerf-slam_amd/pnr/libpnr.so
timeout -k 10 200 python3 bench.py --workload map-points --steps 3 --warmup 1 --no-cpu-baseline --no-gather > gpurun_out/mp17b.log 2>&1 || exit 1
echo "pst $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mp17b.log | head -1)"
python3 -c "
import json
for f in ('gpurun_out/mp17a.log','gpurun_out/mp17b.log'):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, {k:round(v['ms']/d['steps'],2) for k,v in d['kernels'].items()})"
