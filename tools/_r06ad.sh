#!/bin/bash
# 5-slot DMA ring for the delta chain (PNR_BWD_NBUF=5: 160 KiB of LDS): bitwise, kernel timing, room0 A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/lib_ab.py --lib pointnerf-slam_amd/pnr/libpnr.so --out /tmp/a.pt > gpurun_out/r06ad_bit.log 2>&1 || { echo "lib_ab a failed"; tail -20 gpurun_out/r06ad_bit.log; exit 1; }
timeout -k 10 200 python3 tools/lib_ab.py --lib xlibs/libpnr_nb5.so --out /tmp/b.pt --ref /tmp/a.pt >> gpurun_out/r06ad_bit.log 2>&1 || { echo "lib_ab b failed"; tail -20 gpurun_out/r06ad_bit.log; exit 1; }
grep -c "bitwise True" gpurun_out/r06ad_bit.log
O=gpurun_out/r06ad_kb.log; : > $O
for P in 4194304 76032; do for N in base nb5; do
  L=pointnerf-slam_amd/pnr/libpnr.so; [ "$N" != base ] && L=xlibs/libpnr_$N.so
  echo "== $N P=$P" >> $O
  timeout -k 10 120 python3 tools/kbench.py --precision f16x3 --reps 10 --points $P --lib $L >> $O 2>&1 || { echo "FAIL $N"; tail -5 $O; exit 1; }
done; done
grep -E "^==|delta chain" $O
bash tools/_libab.sh nb5 || exit 1
cat gpurun_out/libab.log
