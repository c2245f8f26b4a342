#!/bin/bash
# round-3: the whole GPU suite, then the faithful 1,000-ray iteration under rocprofv3 (kernel trace)
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 750 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gt8.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/gt8.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f1000 -o f -- python3 bench.py --rays 1000 --graph --steps 50 --warmup 3 --no-extras --no-cpu-baseline --no-gather > gpurun_out/f1000.log 2>&1
echo "prof rc=$?"
grep -o '"ms_per_step": [0-9.]*' gpurun_out/f1000.log
