#!/bin/bash
# Round-4 session X: GPU tests and smoke with the scalar slab FMAs, then the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_check.sh
