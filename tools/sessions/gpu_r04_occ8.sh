#!/bin/bash
# Round 4: the walking verify kernel bounded to 64 VGPRs (8 waves per SIMD,
# 7 spilled) against the tree's (68 VGPRs, 7 waves), then the lines whose CPU
# baselines the pinning fix changes.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 700 bash tools/ab_libs.sh "$OUT/ab.jsonl" 3 verify64d,verify wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_occ8/libwireglider_amd.so > "$OUT/ab.txt" 2>&1 || { tail "$OUT/ab.txt"; tail "$OUT/ab.jsonl.err"; exit 1; }
cat "$OUT/ab.txt"
bash tools/gpu_r03.sh "$TAG" bench:verify64d bench:verify bench:config2 bench:gro bench:encap
