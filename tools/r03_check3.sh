#!/bin/bash
# round-3 re-entry check: the GPU test suite, then the default bench line
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gt4.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/gt4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py > gpurun_out/b4.log 2>&1
echo "bench rc=$?"
tail -c 3000 gpurun_out/b4.log
