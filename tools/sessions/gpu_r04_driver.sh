#!/bin/bash
# Round 4: the driver's own invocations — bench.py with no flags (N = 1) and
# two gloo ranks on the one GPU — timed, on the final library.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
S=$(date +%s)
timeout -k 10 600 python3 -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail "$OUT/bench_default.err"; exit 1; }
echo "default bench: $(( $(date +%s) - S )) s"
cut -c1-400 "$OUT/bench_default.json"
bash tools/gpu_r03.sh "$TAG" n2
