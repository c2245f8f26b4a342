#!/bin/bash
# round-3: gather kernel breakdown (rocprofv3), faithful iteration trace with in-place inputs
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g9 -o g -- python3 tools/gather_bench.py --reps 5 > gpurun_out/g9.log 2>&1 || { echo "gather prof rc=$?"; exit 1; }
tail -4 gpurun_out/g9.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f9 -o f -- python3 bench.py --rays 1000 --graph --steps 50 --warmup 3 --no-extras --no-cpu-baseline --no-gather > gpurun_out/f9.log 2>&1 || { echo "faithful prof rc=$?"; exit 1; }
for N in 1000 5000; do
  timeout -k 10 120 python3 bench.py --rays $N --graph --steps 100 --warmup 5 --no-extras --no-cpu-baseline --no-gather > gpurun_out/f${N}c.log 2>&1 || exit $?
  echo "N=$N $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/f${N}c.log)"
done
