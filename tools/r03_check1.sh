#!/bin/bash
# round-3 check: gather microbench, the GPU test suite, faithful-iteration kernel trace
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 150 python -u tools/gather_bench.py > gpurun_out/gb1.log 2>&1 || { echo "gather_bench rc=$?"; exit 1; }
tail -3 gpurun_out/gb1.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/gt2.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f1000b -o f -- python3 bench.py --rays 1000 --graph --steps 50 --warmup 3 --no-extras --no-cpu-baseline --no-gather > gpurun_out/f1000b.log 2>&1
echo "prof rc=$?"
