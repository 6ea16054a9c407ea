#!/bin/bash
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_verify_gates.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_verify.txt" 2>&1 || { tail -30 "$OUT/pytest_verify.txt"; exit 1; }
tail -1 "$OUT/pytest_verify.txt"
for W in verify64d verify64 verify; do
  timeout -k 10 300 python3 -u tools/ab.py $W verify_small=8 verify_small=8,verify_walk_rounds=2 verify_small=7 > "$OUT/ab_$W.json" 2>&1 || { tail "$OUT/ab_$W.json"; exit 1; }
  cat "$OUT/ab_$W.json"
done
echo "session $TAG done"
