#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_w16_tiles.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06z_tests.log 2>&1; rc=$?
tail -8 gpurun_out/r06z_tests.log; exit $rc
