#!/bin/bash
# final: the whole -m gpu suite + smoke, and the auxiliary legs (Tracker, render_img, Mesher grid, configs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_round.sh tests aux
