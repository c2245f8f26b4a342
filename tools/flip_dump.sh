#!/bin/bash
# Diagnostics (GPU box): the end-to-end neural-point gradient tests with PNR_DUMP_GRADS set, so every
# tensor with an element beyond the strict elementwise bound is saved (tests/conftest.py
# maybe_dump_grads) for the offline decision-edge analysis (tools/flip_analysis.py).
#   bash tools/flip_dump.sh <tag>     -> gpurun_out/flips_<tag>/*.npz, gpurun_out/flips_<tag>.log
TAG=${1:-r06}
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PNR_DUMP_GRADS=gpurun_out/flips_${TAG}
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_points.py tests/test_gpu_configs.py -m gpu -v -s --timeout 300 \
  --timeout-method thread -p no:cacheprovider \
  -k 'render_with_points or small_features or tracking_ray_grads or regulation_with_points or c3_office3 or c5_apartment' \
  > gpurun_out/flips_${TAG}.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/flips_${TAG}.log | tail -3
ls gpurun_out/flips_${TAG} 2>/dev/null | head -50
exit $rc
