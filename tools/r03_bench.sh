#!/bin/bash
# round-3: the default bench line (N=1, all extras and CPU baselines)
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > gpurun_out/bench_r03.log 2>&1
echo "bench rc=$?"
tail -c 600 gpurun_out/bench_r03.log
