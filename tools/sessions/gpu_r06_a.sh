#!/bin/bash
# Round 6 evidence, part A: smoke, the whole GPU suite, config 2 (PMC + line
# with the placement-fair CPU baseline + kernel statistics), and the
# multi-thread launch rates on small batches (1 / 4 / 16 threads; 16 threads
# again with one hardware queue per stream).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
bash tools/gpu_r03.sh "$TAG" tests evidence:config2 || exit 1
timeout -k 10 300 python3 -c "
import sys; sys.path[:0] = ['tests', 'oracle']
from pathlib import Path
import test_mt_batch as t
d = Path('$OUT/mt_in'); d.mkdir(exist_ok=True); t.write_inputs(d)" || exit 1
for T in 1 4 16; do
  timeout -k 10 200 tests/cpp/bin/mt_batch "$OUT/mt_in" rate $T 500 small > "$OUT/rate_small_$T.json" 2> "$OUT/rate_small_$T.err" || exit 1
  echo "rate small $T done"
done
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 tests/cpp/bin/mt_batch "$OUT/mt_in" rate 16 500 small > "$OUT/rate_small_16_hwq16.json" \
  2> "$OUT/rate_small_16_hwq16.err" || exit 1
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 tests/cpp/bin/mt_batch "$OUT/mt_in" rate 4 500 small > "$OUT/rate_small_4_hwq16.json" \
  2> "$OUT/rate_small_4_hwq16.err" || exit 1
rm -rf "$OUT/mt_in"
echo "session $TAG done"
