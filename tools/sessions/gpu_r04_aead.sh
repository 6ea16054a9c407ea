#!/bin/bash
# Round 4 AEAD: the pruned kernel set's parity tests (every aead_k, with and
# without the payload-line touch), then same-process A/B of the touch on the
# aead and encap workloads, and same-box alternating-process A/B of the
# 4-waves-per-SIMD register bound (tools/exp/variant_occ4, built with
# -DWG_AEAD_MIN_WAVES=4) against the default build.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_aead.py tests/test_gpu_encap.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > "$OUT/pytest_aead.txt" 2>&1 || { tail -30 "$OUT/pytest_aead.txt"; exit 1; }
tail -1 "$OUT/pytest_aead.txt"
for w in aead encap; do
  timeout -k 10 300 python3 -u tools/ab.py $w aead_pf=0 aead_pf=1 > "$OUT/ab_pf_$w.json" 2> "$OUT/ab_pf_$w.err" || { tail "$OUT/ab_pf_$w.err"; exit 1; }
  cat "$OUT/ab_pf_$w.json"
done
timeout -k 10 900 bash tools/ab_builds.sh "$OUT/ab_occ4.jsonl" 3 wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_occ4/libwireglider_amd.so aead encap > "$OUT/ab_occ4.txt" 2>&1 || { tail "$OUT/ab_occ4.txt"; exit 1; }
cat "$OUT/ab_occ4.txt"
echo "session $TAG done"
