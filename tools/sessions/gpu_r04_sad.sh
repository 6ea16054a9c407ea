#!/bin/bash
# Round 4: 16-bit word sums by v_sad_u16 in the lane paths (L4 lane_sum,
# verify lanes, the AEAD's verify gates) — lane-path parity, then
# alternating-process A/B against the previous build (tools/exp/variant_base).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_l4.py tests/test_gpu_golden_l4.py tests/test_verify_gates.py tests/test_gpu_aead.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
timeout -k 10 900 bash tools/ab_libs.sh "$OUT/ab.jsonl" 3 config4small,verify64d,verify64,config5 wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_base/libwireglider_amd.so > "$OUT/ab.txt" 2>&1 || { tail "$OUT/ab.txt"; tail "$OUT/ab.jsonl.err"; exit 1; }
cat "$OUT/ab.txt"
echo "session $TAG done"
