#!/bin/bash
# Round-4 session B: bench lines at 1 / 2 / 4 frames per launch for c2, c4 and c5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_batch_sweep.sh "c2 c4" "1 2 4" 60 && bash tools/gpu_batch_sweep.sh "c5" "1 2 4" 20
