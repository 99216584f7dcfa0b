#!/bin/bash
# Round-end style run: GPU suite + smoke + default bench (tools/gpu_r04_suite.sh), the two-rank
# launcher rehearsal (tools/gpu_r04_rehearsal.sh), then the PMC passes of one round step on the
# same tree (tools/gpu_r04_pmc.sh, for profiles/r04/pmc/round_traffic.json).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-full}
TAG=$TAG bash tools/gpu_r04_suite.sh && bash tools/gpu_r04_rehearsal.sh && NOBOOT=1 TAG=${TAG}p bash tools/gpu_r04_pmc.sh
