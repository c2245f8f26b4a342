#!/bin/bash
# round-3: gather with wave-aggregated group counters (kernel breakdown + statistics)
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g10 -o g -- python3 tools/gather_bench.py --reps 5 > gpurun_out/g10.log 2>&1 || { echo "gather prof rc=$?"; exit 1; }
grep -v "^[EW]2026" gpurun_out/g10.log | tail -8
