#!/bin/bash
# Round-4 session C: rocprofv3 evidence (kernel trace + stats, serial trace, counter passes) of the
# bench line for c2, c4 and c5 (tools/gpu_profile.sh); summarise here with tools/roofline.py r4.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for c in ${1:-c2 c4 c5}; do
  bash "$REPO/tools/gpu_profile.sh" r4 "$c" || exit $?
done
