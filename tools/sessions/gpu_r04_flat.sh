#!/bin/bash
# Round 4: staged AEAD messages copied out as one flat run when a wave's
# messages are full-size and back to back in memory — AEAD / encap parity,
# then alternating-process A/B against the slot-by-slot copy
# (tools/exp/variant_base).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_aead.py tests/test_gpu_encap.py tests/test_gpu_hostpath.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
timeout -k 10 900 bash tools/ab_libs.sh "$OUT/ab.jsonl" 3 aead,encap wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_base/libwireglider_amd.so > "$OUT/ab.txt" 2>&1 || { tail "$OUT/ab.txt"; tail "$OUT/ab.jsonl.err"; exit 1; }
cat "$OUT/ab.txt"
