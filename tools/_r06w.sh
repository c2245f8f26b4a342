#!/bin/bash
# Adam: 16 elements per thread and pass (55 tickets for the decoder instead of 218): tests, room0 A/B vs HEAD
# bitwise A/B against the previous build (xlibs/libpnr_head.so), room0 timing A/B, room0 kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/lib_ab.py --lib xlibs/libpnr_head.so --out /tmp/a.pt > gpurun_out/r06w_bit.log 2>&1 || { echo "lib_ab a failed"; tail -20 gpurun_out/r06w_bit.log; exit 1; }
timeout -k 10 200 python3 tools/lib_ab.py --lib pointnerf-slam_amd/pnr/libpnr.so --out /tmp/b.pt --ref /tmp/a.pt >> gpurun_out/r06w_bit.log 2>&1 || { echo "lib_ab b failed"; tail -20 gpurun_out/r06w_bit.log; exit 1; }
grep -c "bitwise True" gpurun_out/r06w_bit.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_parity.py tests/test_gpu_sequence.py tests/test_gpu_points.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06w_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06w_tests.log; exit 1; }
tail -1 gpurun_out/r06w_tests.log
bash tools/_libab.sh head || exit 1
cat gpurun_out/libab.log
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r06w_tl -o t -- python3 bench.py --workload room0 --steps 30 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/prof_r06w_tl.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/timeline.py gpurun_out/prof_r06w_tl --period-kernel k_adam_multi
