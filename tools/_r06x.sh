#!/bin/bash
# launch-boundary microbenchmark (tools/micro/launch_gap.hip): which kernel property costs the ~5 us boundaries
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lgap -o g -- ./tools/micro/launch_gap 40 > gpurun_out/lgap.log 2>&1 || { echo "lgap failed"; tail -5 gpurun_out/lgap.log; exit 1; }
python3 tools/micro/launch_gap.py gpurun_out/lgap
