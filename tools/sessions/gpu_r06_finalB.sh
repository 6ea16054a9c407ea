#!/bin/bash
# Round 6 evidence, part B: the other workloads' lines with the
# placement-fair CPU baseline (CPUs dealt over L3 domains, per-worker rates,
# read probe, bound).  usage: gpu_r06_finalB.sh TAG [workload...]
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1; shift
steps=()
for W in "$@"; do steps+=("bench:$W:--no-strong"); done
bash tools/gpu_r03.sh "$TAG" "${steps[@]}" || exit 1
echo "session $TAG done"
