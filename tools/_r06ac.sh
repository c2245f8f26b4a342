#!/bin/bash
# the default bench line at the final commit (room0 traffic from the room0 PMC pass) + smoke
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r06_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python3 bench.py > gpurun_out/r06_bench_final.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r06_bench_final.log; exit 1; }
tail -c 400 gpurun_out/r06_bench_final.log
