#!/bin/bash
# Round profile + bench (GPU box): rocprof kernel stats and traffic passes of the default bench,
# the per-unit traffic json (bench.py reads profiles/r*_traffic.json), then the default bench line.
#   bash tools/round_prof.sh <tag>
set -e
TAG=$1
bash tools/prof_bench.sh $TAG
python3 tools/traffic_json.py gpurun_out/prof_${TAG}_traffic gpurun_out/${TAG}_traffic.json \
  "tools/prof_bench.sh $TAG on MI355X: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline; FETCH_SIZE x2 (gfx950 correction); bytes per unit, mean over the run's launches" > /dev/null
cp gpurun_out/${TAG}_traffic.json profiles/
python3 tools/traffic.py gpurun_out/prof_${TAG}_traffic > gpurun_out/${TAG}_traffic.txt
timeout -k 10 600 python3 bench.py > gpurun_out/bench_${TAG}.log 2>&1
tail -1 gpurun_out/bench_${TAG}.log
