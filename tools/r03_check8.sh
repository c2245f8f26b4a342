#!/bin/bash
# round-3: unrolled 32+12 ray kernels + masked-A weight gradients with features -- the GPU suite,
# then the faithful iteration (N = 1,000 / 5,000) and the neural-point S-map
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 750 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gt10.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/gt10.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for N in 1000 5000; do
  timeout -k 10 120 python3 bench.py --rays $N --graph --steps 100 --warmup 5 --no-extras --no-cpu-baseline --no-gather > gpurun_out/f${N}b.log 2>&1 || exit $?
  echo "N=$N $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/f${N}b.log)"
done
timeout -k 10 200 python3 bench.py --workload map-points --steps 3 --warmup 1 --no-cpu-baseline --no-gather > gpurun_out/mp10.log 2>&1
echo "map-points rc=$? $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mp10.log | head -1)"
timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline --no-gather > gpurun_out/m10.log 2>&1
echo "map rc=$? $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/m10.log | head -1)"
