#!/bin/bash
# round-3: gather kernel breakdown + the re-tightened GPU tests
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g2 -o g -- python3 tools/gather_bench.py --reps 5 > gpurun_out/g2.log 2>&1 || { echo "gather prof rc=$?"; exit 1; }
tail -4 gpurun_out/g2.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_configs.py -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/gt3.log 2>&1
echo "pytest rc=$?"
