#!/bin/bash
# Round 5: the production GSO shape under line-aware cache policies (copy
# only), beside row windows and the production split on the same box.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 tools/exp/bin/gso_tile_copy 20 ${PROBE_MODE:-segs} > "$OUT/seg_copy.jsonl" 2>&1 || { tail "$OUT/seg_copy.jsonl"; exit 1; }
cat "$OUT/seg_copy.jsonl"
timeout -k 10 300 python3 -u tools/ab.py config3 > "$OUT/ab_config3.json" 2>&1 || { tail "$OUT/ab_config3.json"; exit 1; }
cat "$OUT/ab_config3.json"
if [ -n "${AB_R03F:-}" ]; then
  timeout -k 10 900 bash tools/ab_trees.sh "$OUT/ab_r03f.jsonl" 3 config4,config5,config4small tools/exp/r03f_tree . \
    > "$OUT/ab_r03f.txt" 2>&1 || { tail "$OUT/ab_r03f.txt"; exit 1; }
  cat "$OUT/ab_r03f.txt"
fi
echo "session $TAG done"
