#!/bin/bash
# Timing-only ablations of the MLP kernels (GPU box): tools/kbench.py on the in-tree build and on
# experiment builds (tools/xbuild.sh -> xlibs/libpnr_<name>.so), f16x3, 4M points.
#   bash tools/abl_mlp.sh <tag> <name...>      -> gpurun_out/abl_<tag>.log
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/abl_${TAG}.log
: > $O
for N in base "$@"; do
  L=pointnerf-slam_amd/pnr/libpnr.so
  [ "$N" != base ] && L=xlibs/libpnr_$N.so
  echo "== $N" | tee -a $O
  timeout -k 10 120 python3 tools/kbench.py --precision f16x3 --reps 5 --lib $L >> $O 2>&1 || { echo "FAIL $N rc=$?"; tail -5 $O; exit 1; }
done
grep -E "^==|mean_ms|ms/backward|wave " $O
