#!/bin/bash
# round-3: gather kernel breakdown, faithful-iteration trace, the GPU test suite
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g2 -o g -- python3 tools/gather_bench.py --reps 5 > gpurun_out/g2.log 2>&1 || { echo "gather prof rc=$?"; exit 1; }
tail -4 gpurun_out/g2.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f1000c -o f -- python3 bench.py --rays 1000 --graph --steps 50 --warmup 3 --no-extras --no-cpu-baseline --no-gather > gpurun_out/f1000c.log 2>&1 || { echo "faithful prof rc=$?"; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/f1000c.log
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/gt3.log 2>&1
echo "pytest rc=$?"
