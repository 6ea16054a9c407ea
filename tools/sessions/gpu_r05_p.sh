#!/bin/bash
# Round 5 evidence refresh with the round-5 library: PMC traffic, bench line
# and rocprofv3 kernel statistics per workload (part 1: configs 4, 5, 1).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1; shift
bash tools/gpu_r03.sh "$TAG" "$@" || exit 1
echo "session $TAG done"
