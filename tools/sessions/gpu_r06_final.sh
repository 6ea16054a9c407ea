#!/bin/bash
# Round 6 final rehearsal on the final tree: smoke, the whole GPU suite, the
# default bench line (as the driver runs it) and the config 2 PMC + kernel
# statistics of the same tree.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 600 python3 -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail "$OUT/bench_default.err"; exit 1; }
cut -c1-300 "$OUT/bench_default.json"
bash tools/gpu_r03.sh "$TAG" tests evidence:config2 || exit 1
echo "session $TAG done"
