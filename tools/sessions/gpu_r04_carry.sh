#!/bin/bash
# Round 4 AEAD: Poly1305 step with its four column chains independent and
# the carries after them (-DWG_P32_CARRY_LAST=1), with and without LLVM's
# max-ilp scheduler, against the default build (alternating processes).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 1100 bash tools/ab_libs.sh "$OUT/ab.jsonl" 3 aead,encap wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_carry/libwireglider_amd.so tools/exp/variant_carryilp/libwireglider_amd.so \
  tools/exp/variant_ilp/libwireglider_amd.so > "$OUT/ab.txt" 2>&1 || { tail "$OUT/ab.txt"; tail "$OUT/ab.jsonl.err"; exit 1; }
cat "$OUT/ab.txt"
echo "session $TAG done"
