#!/bin/bash
# Round 4: GRO finalize with one packed LDS word per flow (22.5 KB per block,
# 7 waves per SIMD instead of 6) — parity, then alternating-process A/B.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gro_finalize.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
timeout -k 10 900 bash tools/ab_libs.sh "$OUT/ab.jsonl" 4 gro wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_base/libwireglider_amd.so > "$OUT/ab.txt" 2>&1 || { tail "$OUT/ab.txt"; exit 1; }
cat "$OUT/ab.txt"
