#!/bin/bash
# Round 4 AEAD: quarter-round issue rates by rotate form
# (tools/exp/chacha_rate.hip), then same-box alternating-process A/B of the
# library built with LLVM's max-ilp machine scheduler
# (tools/exp/variant_ilp) against the default build on aead and encap.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
hipcc --offload-arch=gfx950 -O3 -o "$OUT/chacha_rate" tools/exp/chacha_rate.hip 2> "$OUT/chacha_build.log" || { tail "$OUT/chacha_build.log"; exit 1; }
timeout -k 10 120 "$OUT/chacha_rate" > "$OUT/chacha_rate.jsonl" 2>&1 || { tail "$OUT/chacha_rate.jsonl"; exit 1; }
cat "$OUT/chacha_rate.jsonl"
timeout -k 10 900 bash tools/ab_builds.sh "$OUT/ab_ilp.jsonl" 3 wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_ilp/libwireglider_amd.so aead encap > "$OUT/ab_ilp.txt" 2>&1 || { tail "$OUT/ab_ilp.txt"; exit 1; }
cat "$OUT/ab_ilp.txt"
echo "session $TAG done"
