#!/bin/bash
# final round-6 profile, part 1: rocprofv3 kernel stats + PMC passes (prof), C3 / C5 (npf)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_round.sh prof npf
