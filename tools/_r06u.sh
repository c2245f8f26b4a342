#!/bin/bash
# final code: the whole -m gpu suite + smoke, room0 timeline + kernel stats, the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_round.sh tests timeline bench || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r06_f1000 -o f -- python3 bench.py --workload room0 --steps 50 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/prof_r06_f1000.log 2>&1 || { echo "room0 stats failed"; exit 1; }
echo FINAL_DONE
