set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 300 python3 bench.py --workload map-points --no-cpu-baseline > gpurun_out/b_mp.json 2> gpurun_out/b_mp.err
cat gpurun_out/b_mp.json
