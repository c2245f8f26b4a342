#!/bin/bash
# round-3: the whole GPU suite (sequence control, one-launch gt max), smoke, faithful timing
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gt18.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/gt18.log
grep -E "control \(fp32|teacher-forced f16x3" gpurun_out/gt18.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke18.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/smoke18.log
for N in 1000 5000; do
  timeout -k 10 120 python3 bench.py --rays $N --graph --steps 100 --warmup 5 --no-extras --no-cpu-baseline --no-gather > gpurun_out/f${N}e.log 2>&1 || exit $?
  echo "N=$N $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/f${N}e.log)"
done
