#!/bin/bash
# Round evidence on one GPU box: for each config, rocprofv3 kernel stats + HBM
# counter passes (tools/gpu_profile.sh), the per-launch traffic merged into
# gpurun_out/traffic.json (tools/traffic.py), then the bench line reading it.
# Copy gpurun_out/{prof_*,traffic.json,bench_*.json} into profiles/<round>/.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r1}"; shift
CFGS=("${@:-c2 c4 c5}")
cd "$REPO"
mkdir -p gpurun_out
cp profiles/r1/traffic.json gpurun_out/traffic.json
for c in ${CFGS[@]}; do
  bash tools/gpu_profile.sh "$TAG" "$c" || exit $?
  python3 tools/traffic.py "gpurun_out/prof_${TAG}_${c}" "$c" gpurun_out/traffic.json || exit $?
done
for c in ${CFGS[@]}; do
  timeout -k 10 600 python3 bench.py --config "$c" --traffic gpurun_out/traffic.json > "gpurun_out/bench_$c.json" 2> "gpurun_out/bench_$c.err"; rc=$?
  echo "bench $c=$rc"; [ $rc -eq 0 ] || exit $rc
done
