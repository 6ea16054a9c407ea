#!/bin/bash
# Round 4: the walking descriptor kernels (l4_small = 6, verify_small = 8)
# against the split / wave / compacting kernels; parity first.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_l4.py tests/test_verify_gates.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "desc_random or desc_small or verify_parity or size_gate or interleaved" \
  > "$OUT/pytest_walk.txt" 2>&1 || { tail -30 "$OUT/pytest_walk.txt"; exit 1; }
tail -1 "$OUT/pytest_walk.txt"
bash tools/gpu_r03.sh "$TAG" ab:config4small:l4_small=5:l4_small=6:l4_small=6,l4_unroll=4 \
  ab:config5:l4_small=5:l4_small=6:l4_small=6,l4_unroll=4 ab:config4:l4_small=5:l4_small=6:l4_small=6,l4_unroll=4 || exit 1
timeout -k 10 400 python3 -u tools/verify_ab.py verify_small=0 verify_small=7 verify_small=8 verify_small=8,verify_occ=0 \
  verify_small=8,verify_dm=2 > "$OUT/verify_ab.json" 2>&1 || { tail -20 "$OUT/verify_ab.json"; exit 1; }
tail -1 "$OUT/verify_ab.json" | cut -c1-3000
echo "session $TAG done"
