#!/bin/bash
# final round-6 profile, part 2: room0 timeline, the default bench line, the neural-point S-map kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_round.sh timeline bench mpstats
