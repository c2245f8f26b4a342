#!/bin/bash
# HIP runtime knobs vs the room0 iteration's launch boundaries (graph replay): alternating runs
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
O=gpurun_out/r06y_ab.log; : > $O
run() {  # run <tag> <env...>
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --workload room0 --steps 200 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/r06y_$tag.json 2>gpurun_out/r06y_err.log || { echo "bench failed $tag"; tail -5 gpurun_out/r06y_err.log; exit 1; }
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06y_$tag.json | head -1)" | tee -a $O
}
for r in 1 2; do
  run base PNR_NOOP=1
  run pktcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
  run pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run devkarg0 HIP_FORCE_DEV_KERNARG=0
  run devkarg1 HIP_FORCE_DEV_KERNARG=1
done
