#!/bin/bash
# Round-3 end check at the final code: the whole -m gpu suite and smoke()
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final2_gpu_tests.log 2>&1
tail -3 gpurun_out/final2_gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2_smoke.log 2>&1
echo smoke ok
