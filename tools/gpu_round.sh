#!/bin/bash
# GPU-box driver for one round's measurements (replaces the per-call r0N_*.sh scripts).
#   bash tools/gpu_round.sh <step> [<step> ...]      steps run in order; the first failure stops the call
# Steps (each under its own time limit; logs under gpurun_out/<TAG>_*, TAG from $PNR_TAG, default r04):
#   tests       the whole -m gpu suite, then __graft_entry__.smoke()    (pytest failures stop the call)
#   test:<k>    the -m gpu tests matching -k <k>
#   bench       the default bench line (N=1, every extra and CPU baseline)
#   quick       the S-map line alone (no extras / CPU baseline / gather)
#   faithful    the room0 Mapper iteration legs (graph replay) alone
#   points      the neural-point S-map alone
#   gather      tools/gather_bench.py (forward + backward gather timing)
#   aux         the auxiliary benches: Tracker, render_img, Mesher grid, configs C3 / C5
#   timeline    rocprofv3 kernel trace of the replayed room0 iteration -> ${TAG}_room0_timeline.txt
#   pmcsearch   the gather search's stall counters (tools/pmc_search.sh)
#   mpstats     rocprofv3 kernel stats of the neural-point S-map (--workload map-points)
#   npf         the faithful-size neural-point iterations C3 / C5 (tools/np_faithful.py) + their kernel stats
#   prof        the round profile: rocprofv3 kernel stats + FETCH/WRITE and MFMA-busy PMC passes
#               (tools/prof_round.sh), the gather's traffic passes and kernel stats, the faithful
#               iteration's kernel stats
set -o pipefail
TAG=${PNR_TAG:-r06}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/${TAG}

run() {  # run <seconds> <log> <cmd...>: stop the whole call on a non-zero status
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "FAILED rc=$rc: $*"; tail -25 "$log"; exit $rc
  fi
}

for step in "$@"; do
  case $step in
    tests)
      run 1000 ${O}_gpu_tests.log python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        -p no:cacheprovider
      tail -2 ${O}_gpu_tests.log
      run 200 ${O}_smoke.log python3 -c "import __graft_entry__ as g; g.smoke()"
      echo "smoke ok" ;;
    test:*)
      K="${step#test:}"; L="${O}_gpu_tests_${K//[^A-Za-z0-9_]/_}.log"
      run 900 "$L" python3 -u -m pytest tests -m gpu -x -v --timeout 300 \
        --timeout-method thread -p no:cacheprovider -k "$K"
      tail -3 "$L" ;;
    bench)
      run 600 ${O}_bench.log python3 bench.py
      tail -c 300 ${O}_bench.log; echo ;;
    quick)
      run 300 ${O}_quick.log python3 bench.py --workload map --steps 5 --warmup 2 --no-extras --no-cpu-baseline --no-gather
      grep -o '"value": [0-9.]*, "unit": "rays/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' ${O}_quick.log
      grep -o '"frac": [0-9.]*' ${O}_quick.log | head -1 ;;
    faithful)
      run 300 ${O}_faithful.log python3 bench.py --workload room0 --steps 100 --warmup 5 --no-cpu-baseline --no-extras
      tail -c 400 ${O}_faithful.log; echo ;;
    points)
      run 300 ${O}_points.log python3 bench.py --workload map-points --steps 3 --warmup 1 --no-cpu-baseline --no-gather
      grep -o '"ms_per_step": [0-9.]*' ${O}_points.log | head -1 ;;
    gather)
      run 300 ${O}_gather.log python3 tools/gather_bench.py
      tail -8 ${O}_gather.log ;;
    timeline)
      run 200 gpurun_out/prof_${TAG}_tl.log rocprofv3 --kernel-trace --output-format csv \
        -d gpurun_out/prof_${TAG}_tl -o t -- python3 bench.py --workload room0 --steps 30 --warmup 3 --no-extras \
        --no-cpu-baseline
      python3 tools/timeline.py gpurun_out/prof_${TAG}_tl --period-kernel k_adam_multi > ${O}_room0_timeline.txt
      cat ${O}_room0_timeline.txt ;;
    pmcsearch)
      bash tools/pmc_search.sh ${TAG} > ${O}_pmcsearch.log 2>&1 || { echo "FAILED pmcsearch"; tail -5 ${O}_pmcsearch.log; exit 1; }
      tail -12 ${O}_pmcsearch.log ;;
    npf)
      run 200 ${O}_c3.log python3 tools/np_faithful.py --case C3 --iters 50
      run 200 ${O}_c3_bf16.log python3 tools/np_faithful.py --case C3 --iters 50 --precision bf16
      tail -1 ${O}_c3_bf16.log
      run 200 ${O}_c5.log python3 tools/np_faithful.py --case C5 --iters 30
      tail -1 ${O}_c3.log; tail -1 ${O}_c5.log
      run 300 gpurun_out/prof_${TAG}_c3.log rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/prof_${TAG}_c3 -o c3 -- python3 tools/np_faithful.py --case C3 --iters 30
      run 300 gpurun_out/prof_${TAG}_c5.log rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/prof_${TAG}_c5 -o c5 -- python3 tools/np_faithful.py --case C5 --iters 20
      echo npf-prof ;;
    mpstats)
      run 300 gpurun_out/prof_${TAG}_mp.log rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/prof_${TAG}_mp -o mp -- python3 bench.py --workload map-points --steps 3 --warmup 1 \
        --no-cpu-baseline --no-gather
      echo mpstats ;;
    aux)
      run 200 ${O}_track.json python3 tools/track_bench.py
      run 200 ${O}_render.json python3 tools/render_bench.py
      run 200 ${O}_mesh.json python3 tools/mesh_eval_bench.py
      run 400 ${O}_configs.json python3 tools/config_bench.py
      echo "aux ok" ;;
    prof)
      bash tools/prof_round.sh ${TAG} || exit $?
      for C in FETCH_SIZE WRITE_SIZE; do
        run 200 gpurun_out/prof_${TAG}_g$C.log rocprofv3 --kernel-trace --pmc $C --output-format csv \
          -d gpurun_out/prof_${TAG}_gtraffic -o $C -- python3 tools/gather_bench.py --reps 2
      done
      run 200 gpurun_out/prof_${TAG}_gb.log rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/prof_${TAG}_gather -o gb -- python3 tools/gather_bench.py
      run 200 gpurun_out/prof_${TAG}_f1000.log rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/prof_${TAG}_f1000 -o f -- python3 bench.py --workload room0 --steps 50 --warmup 3 --no-extras \
        --no-cpu-baseline
      echo "ROUND_PROF_DONE" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
