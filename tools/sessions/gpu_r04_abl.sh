#!/bin/bash
# Round 4: timing-only AEAD ablations (wrong tags; never in the library):
# Poly1305 steps replaced by an XOR (variant_nopoly), the suffix-product tree
# skipped (variant_nostree) — how much of the encrypt kernel's time each
# serial part holds.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 bash tools/ab_libs.sh "$OUT/ab.jsonl" 3 aead wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_nopoly/libwireglider_amd.so tools/exp/variant_nostree/libwireglider_amd.so > "$OUT/ab.txt" 2>&1 || { tail "$OUT/ab.txt"; tail "$OUT/ab.jsonl.err"; exit 1; }
cat "$OUT/ab.txt"
