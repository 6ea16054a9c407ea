#!/bin/bash
# Round 4 full-tree session: smoke, the whole GPU suite, then the bench lines
# (PMC + line + rocprofv3 kernel stats from the same box for the main ones).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
shift
mkdir -p "gpurun_out/$TAG"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "gpurun_out/$TAG/smoke.txt" 2>&1 || { tail -20 "gpurun_out/$TAG/smoke.txt"; exit 1; }
tail -1 "gpurun_out/$TAG/smoke.txt"
bash tools/gpu_r03.sh "$TAG" "$@"
