#!/bin/bash
# round-3: the changed neural-point / config tests first, then the whole GPU suite, the bench line,
# and the gather kernels under rocprofv3
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_configs.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gt5a.log 2>&1
rc=$?
echo "pytest(points,configs) rc=$rc"; tail -3 gpurun_out/gt5a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_points.py --deselect tests/test_gpu_configs.py > gpurun_out/gt5b.log 2>&1
rc=$?
echo "pytest(rest) rc=$rc"; tail -3 gpurun_out/gt5b.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py > gpurun_out/b5.log 2>&1
echo "bench rc=$?"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g5 -o g -- python3 tools/gather_bench.py --reps 5 > gpurun_out/g5.log 2>&1
echo "gather prof rc=$?"
