#!/bin/bash
# round-3: dWc_3 on a rebuilt dL/dh4 (neural-point tests + map-points bench), then the round profile
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_configs.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gt16.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/gt16.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python3 bench.py --workload map-points --steps 3 --warmup 1 --no-cpu-baseline --no-gather > gpurun_out/mp16.log 2>&1
echo "map-points rc=$? $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mp16.log | head -1)"
bash tools/round_r03.sh r03
