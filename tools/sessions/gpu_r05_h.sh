#!/bin/bash
# Round 5: the split's one-segment-per-wave geometries (the copy probe's
# fastest segment shape) against the default, one process.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/ab.py config3 gso_occ=0 gso_occ=3 gso_occ=4 gso_occ=2 gso_occ=3,gso_groups=1 gso_occ=4,gso_spw=3 \
  > "$OUT/ab_config3.json" 2>&1 || { tail "$OUT/ab_config3.json"; exit 1; }
cat "$OUT/ab_config3.json"
echo "session $TAG done"
