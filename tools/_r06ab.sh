#!/bin/bash
# PMC traffic of the room0 iteration (separate FETCH_SIZE / WRITE_SIZE passes): the headline kernel's bytes per launch
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/prof_r06_r0traffic -o $C -- \
    python3 bench.py --workload room0 --steps 10 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/prof_r06_r0$C.log 2>&1 || { echo "FAILED $C"; tail -5 gpurun_out/prof_r06_r0$C.log; exit 1; }
  echo $C
done
python3 tools/traffic_json.py gpurun_out/prof_r06_r0traffic gpurun_out/r06_r0traffic.json "room0" --mlp-points=76032
