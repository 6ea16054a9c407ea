#!/bin/bash
# Round 4: the split kernel's wave role one long packet at a time (64 VGPRs,
# 8 waves per SIMD) against two (74, 6) — alternating processes.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 bash tools/ab_libs.sh "$OUT/ab.jsonl" 3 config4small,config4,config5 wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_q1/libwireglider_amd.so > "$OUT/ab.txt" 2>&1 || { tail "$OUT/ab.txt"; exit 1; }
cat "$OUT/ab.txt"
