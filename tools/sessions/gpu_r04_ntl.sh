#!/bin/bash
# Round 4: the full GSO split's payload loads non-temporal (variant_ntl)
# against default-policy loads — alternating processes on config 3 / 3udp.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 bash tools/ab_libs.sh "$OUT/ab.jsonl" 3 config3,config3udp wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_ntl/libwireglider_amd.so > "$OUT/ab.txt" 2>&1 || { tail "$OUT/ab.txt"; exit 1; }
cat "$OUT/ab.txt"
