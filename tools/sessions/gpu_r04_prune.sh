#!/bin/bash
# Round 4: the pruned library (rejected variants removed, verify default with
# the walking kernel, capture-safe): the affected GPU tests, the verify A/B and
# the first-call probe.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_l4.py tests/test_verify_gates.py tests/test_gro_finalize.py \
  tests/test_gpu_golden_l4.py tests/test_gpu_hostpath.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > "$OUT/pytest_prune.txt" 2>&1 || { tail -30 "$OUT/pytest_prune.txt"; exit 1; }
tail -1 "$OUT/pytest_prune.txt"
timeout -k 10 300 python3 -u tools/verify_first_call.py > "$OUT/first_call.json" 2>&1 || { tail -20 "$OUT/first_call.json"; exit 1; }
tail -1 "$OUT/first_call.json"
timeout -k 10 400 python3 -u tools/verify_ab.py > "$OUT/verify_ab.json" 2>&1 || { tail -20 "$OUT/verify_ab.json"; exit 1; }
echo "session $TAG done"
