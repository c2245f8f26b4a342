#!/bin/bash
# round-3: gather (two-row feature rounds, aggregated group counters): neural-point tests + bench
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_crafted.py tests/test_gpu_edges.py tests/test_gpu_configs.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gt13.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/gt13.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 150 python3 tools/gather_bench.py --reps 10 > gpurun_out/g13.log 2>&1; grep "k_gather" gpurun_out/g13.log
