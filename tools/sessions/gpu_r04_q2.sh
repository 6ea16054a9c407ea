#!/bin/bash
# Round 4: the split descriptor kernel's wave role issuing 2 packets at a
# time instead of 4 (U = 8: 74 VGPRs, 6 waves per SIMD; U = 4: 54, 8) against
# the tree's (94 / 74) — alternating processes, at l4_unroll 8 and 4.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 bash tools/ab_libs.sh "$OUT/ab_u8.jsonl" 3 config4small,config4,config5 wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_q2/libwireglider_amd.so > "$OUT/ab_u8.txt" 2>&1 || { tail "$OUT/ab_u8.txt"; exit 1; }
cat "$OUT/ab_u8.txt"
WG_L4_UNROLL=4 timeout -k 10 900 bash tools/ab_libs.sh "$OUT/ab_u4.jsonl" 3 config4small,config4,config5 wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_q2/libwireglider_amd.so > "$OUT/ab_u4.txt" 2>&1 || { tail "$OUT/ab_u4.txt"; exit 1; }
cat "$OUT/ab_u4.txt"
