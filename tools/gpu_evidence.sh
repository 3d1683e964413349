#!/bin/bash
# Round evidence on one GPU box: for each config the rocprofv3 trace + counter
# passes of tools/gpu_profile.sh, then the bench line. Afterwards, here:
#   python tools/roofline.py <tag> <cfgs...>   (profiles/<tag>/, counters.json)
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r2}"; shift
CFGS=("${@:-c2 c4 c5}")
cd "$REPO"
mkdir -p gpurun_out
for c in ${CFGS[@]}; do
  bash tools/gpu_profile.sh "$TAG" "$c" || exit $?
done
