#!/bin/bash
# round-3: per-point B scale in the hidden weight-gradient GEMMs -- the changed gradient tests, then
# the S-map bench line (weight-gradient time)
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_points.py tests/test_gpu_precision.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gt7.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -6 gpurun_out/gt7.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python3 bench.py --no-extras --no-cpu-baseline --no-gather > gpurun_out/b7.log 2>&1
echo "bench rc=$?"
tail -c 1500 gpurun_out/b7.log
