#!/bin/bash
# Round 4: split-role verify at 8 waves/SIMD (verify_small = 10); parity first.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_golden_l4.py tests/test_verify_gates.py tests/test_gpu_hostpath.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "golden or reference or verify_parity or size_gate or interleaved or build_failure or small_reads" \
  > "$OUT/pytest_vsplit.txt" 2>&1 || { tail -30 "$OUT/pytest_vsplit.txt"; exit 1; }
tail -1 "$OUT/pytest_vsplit.txt"
timeout -k 10 400 python3 -u tools/verify_ab.py verify_small=0 verify_small=7 verify_small=8,verify_occ=0 verify_small=10 \
  verify_small=10,verify_occ=0 > "$OUT/verify_ab.json" 2>&1 || { tail -20 "$OUT/verify_ab.json"; exit 1; }
echo "session $TAG done"
