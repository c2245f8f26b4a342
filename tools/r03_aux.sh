#!/bin/bash
# round-3: the auxiliary benches (Tracker, render_img, Mesher grid, configs C3 / C5) at the round's code
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/track_bench.py > gpurun_out/r03_track.json 2> gpurun_out/r03_track.err || { echo "track rc=$?"; exit 1; }
tail -c 400 gpurun_out/r03_track.json; echo
timeout -k 10 200 python3 tools/render_bench.py > gpurun_out/r03_render.json 2> gpurun_out/r03_render.err || { echo "render rc=$?"; exit 1; }
tail -c 400 gpurun_out/r03_render.json; echo
timeout -k 10 200 python3 tools/mesh_eval_bench.py > gpurun_out/r03_mesh.json 2> gpurun_out/r03_mesh.err || { echo "mesh rc=$?"; exit 1; }
tail -c 400 gpurun_out/r03_mesh.json; echo
timeout -k 10 300 python3 tools/config_bench.py > gpurun_out/r03_configs.json 2> gpurun_out/r03_configs.err || { echo "configs rc=$?"; exit 1; }
tail -c 800 gpurun_out/r03_configs.json; echo
