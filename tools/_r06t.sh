#!/bin/bash
# float4 partial reduction (k_part_reduce_multi): bitwise A/B against PNR_REDUCE_VEC=0, room0 timing A/B, timeline
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
L=pointnerf-slam_amd/pnr/libpnr.so
PNR_REDUCE_VEC=0 timeout -k 10 200 python3 tools/lib_ab.py --lib $L --out /tmp/a.pt > gpurun_out/r06t_bit.log 2>&1 || { echo "lib_ab a failed"; tail -20 gpurun_out/r06t_bit.log; exit 1; }
timeout -k 10 200 python3 tools/lib_ab.py --lib $L --out /tmp/b.pt --ref /tmp/a.pt >> gpurun_out/r06t_bit.log 2>&1 || { echo "lib_ab b failed"; tail -20 gpurun_out/r06t_bit.log; exit 1; }
grep -c "bitwise True" gpurun_out/r06t_bit.log
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_parity.py tests/test_gpu_points.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06t_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06t_tests.log; exit 1; }
tail -1 gpurun_out/r06t_tests.log
O=gpurun_out/r06t_ab.log; : > $O
for r in 1 2 3; do for F in 1 0; do
  PNR_REDUCE_VEC=$F timeout -k 10 200 python3 bench.py --workload room0 --steps 200 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/r06t_$F.json 2>gpurun_out/r06t_err.log || { echo "bench failed"; tail -5 gpurun_out/r06t_err.log; exit 1; }
  echo "$r vec=$F $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06t_$F.json | head -1)" >> $O
done; done
cat $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r06t_tl -o t -- python3 bench.py --workload room0 --steps 30 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/prof_r06t_tl.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/timeline.py gpurun_out/prof_r06t_tl --period-kernel k_adam_multi
