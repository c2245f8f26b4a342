#!/bin/bash
# Round profile (GPU box): rocprofv3 kernel-trace stats of the S-map (default) and S-fwd bench
# commands, then separate --pmc passes (one counter group per run, MI355X_MICROARCH.md):
#   FETCH_SIZE, WRITE_SIZE           HBM bytes of the S-map step (FETCH x2: gfx950 correction)
#   SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE + SQ_BUSY_CYCLES   MFMA-busy of S-map and S-fwd
#   bash tools/prof_round.sh <tag>      -> gpurun_out/prof_<tag>*/ (copy the summaries into profiles/)
TAG=${1:-r02}
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
set -e
MAP="python3 bench.py --workload map --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-gather"
FWD="python3 bench.py --workload fwd --steps 5 --warmup 1 --no-cpu-baseline --no-extras"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o map -- \
  $MAP > gpurun_out/prof_${TAG}_map.log 2>&1
echo map-trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_fwd -o fwd -- \
  $FWD > gpurun_out/prof_${TAG}_fwd.log 2>&1
echo fwd-trace
ONE="python3 bench.py --workload map --steps 1 --warmup 0 --no-cpu-baseline --no-extras --no-gather"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/prof_${TAG}_traffic -o $C -- \
    $ONE > gpurun_out/prof_${TAG}_$C.log 2>&1
  echo $C
done
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES \
  --output-format csv -d gpurun_out/prof_${TAG}_mfma -o map -- $ONE > gpurun_out/prof_${TAG}_mfma_map.log 2>&1
echo mfma-map
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES \
  --output-format csv -d gpurun_out/prof_${TAG}_mfma_fwd -o fwd -- \
  python3 bench.py --workload fwd --steps 2 --warmup 0 --no-cpu-baseline --no-extras \
  > gpurun_out/prof_${TAG}_mfma_fwd.log 2>&1
echo PROF_DONE
