#!/bin/bash
# Round 5: ping-pong long packets in the split kernel's wave role (next
# packet's issue loads before the current one is finished), U = 5 / 7 rest
# loads, against the library; config 4 / 4-small / 5, alternating processes.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 bash tools/ab_libs.sh "$OUT/ab_pp.jsonl" 3 config4,config4small,config5 \
  "$ROOT/wireglider_amd/lib/libwireglider_amd.so" tools/exp/variant_pp5/libwireglider_amd.so tools/exp/variant_pp7/libwireglider_amd.so \
  > "$OUT/ab_pp.txt" 2>&1 || { tail "$OUT/ab_pp.txt"; exit 1; }
cat "$OUT/ab_pp.txt"
echo "session $TAG done"
