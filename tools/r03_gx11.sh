#!/bin/bash
# Gather A/B: in-tree (fill-first probe, strided scatter, paired collision-free search loop) vs
# xlibs/libpnr_sserial.so (same, old search loop) vs xlibs/libpnr_serial.so (round-3 start)
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_points.py tests/test_gpu_crafted.py > gpurun_out/gx11_tests.log 2>&1
tail -2 gpurun_out/gx11_tests.log
PNR_LIB_PATH=$GRAFT_REPO_ROOT/xlibs/libpnr_r4w3.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_points.py tests/test_gpu_crafted.py > gpurun_out/gx11_tests_hpf.log 2>&1
tail -2 gpurun_out/gx11_tests_hpf.log
for i in 1 2; do
  for L in pointnerf-slam_amd/pnr/libpnr.so xlibs/libpnr_r4w3.so xlibs/libpnr_serial.so; do
    echo "== $L"
    timeout -k 10 150 python3 tools/gather_bench.py --reps 10 --lib $L 2>&1 | grep -E "k_gather "
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gx11 -o gb -- \
  python3 tools/gather_bench.py > gpurun_out/prof_gx11_gb.log 2>&1
echo GX_DONE
