#!/bin/bash
# 4-wave (64-point tile) k_mlp_fwd16w for small batches: forward/gradient tests, room0 A/B vs PNR_W16_NW4=0
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_precision.py tests/test_gpu_determinism.py tests/test_gpu_edges.py tests/test_gpu_crafted.py tests/test_gpu_points_forced.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06l_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06l_tests.log; exit 1; }
tail -2 gpurun_out/r06l_tests.log
O=gpurun_out/r06l_ab.log; : > $O
for r in 1 2 3; do for F in 1 0; do
  PNR_W16_NW4=$F timeout -k 10 200 python3 bench.py --workload room0 --steps 200 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/r06l_$F.json 2>gpurun_out/r06l_err.log || { echo "bench failed"; tail -5 gpurun_out/r06l_err.log; exit 1; }
  echo "$r nw4=$F $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06l_$F.json | head -1)" >> $O
done; done
cat $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r06l_tl -o t -- python3 bench.py --workload room0 --steps 30 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/prof_r06l_tl.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/timeline.py gpurun_out/prof_r06l_tl --period-kernel k_adam_multi
