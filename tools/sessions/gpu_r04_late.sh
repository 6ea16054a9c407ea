#!/bin/bash
# Round 4 AEAD: a K = 3 lane's third ChaCha20 block computed beside the powers
# of r (-DWG_AEAD_TRI_LATE=1: the multiply chains fill its issue gaps) against
# the default build, alternating processes; then the parity tests on it.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 bash tools/ab_libs.sh "$OUT/ab.jsonl" 3 aead,encap wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_late/libwireglider_amd.so > "$OUT/ab.txt" 2>&1 || { tail "$OUT/ab.txt"; tail "$OUT/ab.jsonl.err"; exit 1; }
cat "$OUT/ab.txt"
WG_LIB=tools/exp/variant_late/libwireglider_amd.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_aead.py tests/test_gpu_encap.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > "$OUT/pytest_late.txt" 2>&1 || { tail -30 "$OUT/pytest_late.txt"; exit 1; }
tail -1 "$OUT/pytest_late.txt"
echo "session $TAG done"
