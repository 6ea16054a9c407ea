#!/bin/bash
# Round 5: copy ceilings of the GSO access shapes (row windows of 1-8 KiB,
# segment tiles) beside the production split on the same box; the drop-in at
# 1 / 16 threads (thread-private accumulators).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 tools/exp/bin/gso_tile_copy 20 > "$OUT/tile_copy.jsonl" 2>&1 || { tail "$OUT/tile_copy.jsonl"; exit 1; }
cat "$OUT/tile_copy.jsonl"
timeout -k 10 300 python3 -u tools/ab.py config3 gso_rows=0 > "$OUT/ab_config3.json" 2>&1 || { tail "$OUT/ab_config3.json"; exit 1; }
cat "$OUT/ab_config3.json"




nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c "import os; print(len(os.sched_getaffinity(0)))"
echo "session $TAG done"
