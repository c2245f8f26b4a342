#!/bin/bash
# round-3: gather search with per-lane hit buffers -- neural-point tests, then A/B against the
# network-per-candidate build
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_crafted.py tests/test_gpu_edges.py tests/test_gpu_configs.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gt15.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/gt15.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 150 python3 tools/gather_bench.py --reps 10 2>&1 | grep "k_gather " || exit 1
cp pointnerf-slam_amd/pnr/libpnr.so /tmp/libpnr_intree.so
cp xlibs/libpnr_nohb.so pointnerf-slam_amd/pnr/libpnr.so && echo nohb && timeout -k 10 150 python3 tools/gather_bench.py --reps 10 2>&1 | grep "k_gather " || exit 1
cp /tmp/libpnr_intree.so pointnerf-slam_amd/pnr/libpnr.so && echo hb-again && timeout -k 10 150 python3 tools/gather_bench.py --reps 10 2>&1 | grep "k_gather "
