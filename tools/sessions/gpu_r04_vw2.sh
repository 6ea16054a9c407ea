#!/bin/bash
# Round 4: the walking verify kernel walking its long packets 2 at a time
# instead of 4 (48 VGPRs, 8 waves per SIMD, against 68 / 7) — A/B on the
# all-small batch (the walking kernel's default case) and the first call on
# fresh streams (tools/verify_first_call.py, both builds).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 bash tools/ab_libs.sh "$OUT/ab.jsonl" 3 verify64d wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_vw2/libwireglider_amd.so > "$OUT/ab.txt" 2>&1 || { tail "$OUT/ab.txt"; exit 1; }
cat "$OUT/ab.txt"
for L in wireglider_amd/lib/libwireglider_amd.so tools/exp/variant_vw2/libwireglider_amd.so; do
  WG_LIB=$L timeout -k 10 300 python3 -u tools/verify_first_call.py > "$OUT/first_$(basename $(dirname $L)).json" 2>&1 || { tail "$OUT/first_$(basename $(dirname $L)).json"; exit 1; }
  echo "$L"; tail -1 "$OUT/first_$(basename $(dirname $L)).json" | cut -c1-600
done
