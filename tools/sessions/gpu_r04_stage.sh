#!/bin/bash
# Round 4 AEAD: encrypt's messages assembled in LDS and written in whole lines
# (aead_stage = 1) — parity tests, same-process A/B against lane stores, and
# the write bytes of both (rocprofv3 WRITE_SIZE / FETCH_SIZE passes).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_aead.py tests/test_gpu_encap.py tests/test_gpu_hostpath.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > "$OUT/pytest_aead.txt" 2>&1 || { tail -30 "$OUT/pytest_aead.txt"; exit 1; }
tail -1 "$OUT/pytest_aead.txt"
for w in aead encap; do
  timeout -k 10 300 python3 -u tools/ab.py $w aead_stage=0 aead_stage=1 > "$OUT/ab_stage_$w.json" 2> "$OUT/ab_stage_$w.err" || { tail "$OUT/ab_stage_$w.err"; exit 1; }
  cat "$OUT/ab_stage_$w.json"
done
for v in 0 1; do
  WG_AEAD_STAGE=$v timeout -k 10 300 bash tools/counters.sh "$OUT/pmc_stage$v" aead aead_kernel "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE" "WRITE_SIZE" > "$OUT/pmc_stage$v.log" 2>&1 || { tail -20 "$OUT/pmc_stage$v.log"; exit 1; }
  grep -A8 '"kernels"' "$OUT/pmc_stage$v/summary.json"
done
echo "session $TAG done"
