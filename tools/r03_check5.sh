#!/bin/bash
# round-3 re-entry: the whole GPU suite, then the default bench line
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 750 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gt6.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/gt6.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py > gpurun_out/b6.log 2>&1
echo "bench rc=$?"
tail -c 2500 gpurun_out/b6.log
