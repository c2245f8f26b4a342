#!/bin/bash
# Experiment build: libpnr.so with extra defines -> xlibs/libpnr_<name>.so (git-ignored; ships with gpurun)
#   bash tools/xbuild.sh <name> "-DPNR_EXP_FOO ..."
set -e
NAME=$1; DEFS=$2
cd "$(dirname "$0")/../pointnerf-slam_amd"
OBJ=/tmp/xb_$NAME; mkdir -p $OBJ ../xlibs
FLAGS="-O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=gfx950 -Wall -Wno-unused-function -I/opt/rocm/include $DEFS"
pids=()
for f in csrc/*.hip csrc/capi.cpp; do
  /opt/rocm/bin/hipcc $FLAGS -x hip -c $f -o $OBJ/$(basename $f).o & pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 $OBJ/*.o -shared -o ../xlibs/libpnr_$NAME.so
echo built xlibs/libpnr_$NAME.so
