#!/bin/bash
# fused fc_c weight-gradient GEMMs (FC): neural-point gradient tests, then A/B against PNR_WGRAD_FC_FUSE=0
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_points.py tests/test_gpu_points_forced.py tests/test_gpu_configs.py tests/test_gpu_determinism.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06k_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06k_tests.log; exit 1; }
tail -2 gpurun_out/r06k_tests.log
O=gpurun_out/r06k_ab.log; : > $O
for r in 1 2; do for F in 1 0; do
  echo "== fuse=$F round $r" >> $O
  PNR_WGRAD_FC_FUSE=$F timeout -k 10 200 python3 tools/np_faithful.py --case C5 --iters 30 --mode graph 2>&1 | tail -1 >> $O || { echo "C5 failed"; tail -5 $O; exit 1; }
  PNR_WGRAD_FC_FUSE=$F timeout -k 10 200 python3 tools/np_faithful.py --case C3 --iters 50 --mode graph 2>&1 | tail -1 >> $O || { echo "C3 failed"; tail -5 $O; exit 1; }
  PNR_WGRAD_FC_FUSE=$F timeout -k 10 300 python3 bench.py --workload map-points --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/r06k_mp_$F.json 2>gpurun_out/r06k_err.log || { echo "mp failed"; tail -5 gpurun_out/r06k_err.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06k_mp_$F.json | head -1 >> $O
done; done
cat $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r06k_c5 -o c5 -- python3 tools/np_faithful.py --case C5 --iters 20 --mode graph > gpurun_out/prof_r06k_c5.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
