#!/bin/bash
# Round 4 L4: the split-role kernel's lane-role wave rotated over the block's
# four waves (block b: wave b % 4) — parity tests, then alternating-process
# A/B against the previous l4csum.hip (tools/exp/variant_base).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_l4.py tests/test_gpu_golden_l4.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > "$OUT/pytest_l4.txt" 2>&1 || { tail -30 "$OUT/pytest_l4.txt"; exit 1; }
tail -1 "$OUT/pytest_l4.txt"
timeout -k 10 1000 bash tools/ab_libs.sh "$OUT/ab.jsonl" 3 config4small,config4,config5 wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_base/libwireglider_amd.so > "$OUT/ab.txt" 2>&1 || { tail "$OUT/ab.txt"; tail "$OUT/ab.jsonl.err"; exit 1; }
cat "$OUT/ab.txt"
echo "session $TAG done"
