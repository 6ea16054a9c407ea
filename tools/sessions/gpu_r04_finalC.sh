#!/bin/bash
# Round 4 final evidence, part C (after the flat copy-out): SQ counters of the
# AEAD and encap kernels (profiles/valu_{aead,encap}.json), then their PMC +
# bench line + kernel statistics.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for W in aead encap; do
  timeout -k 10 400 bash tools/counters.sh "$OUT/sq_$W" $W aead_kernel \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
    "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH" \
    "GRBM_GUI_ACTIVE GRBM_COUNT" > "$OUT/sq_$W.log" 2>&1 || { tail -20 "$OUT/sq_$W.log"; exit 1; }
  timeout -k 10 300 python3 -u bench.py --workload $W --steps 20 --no-cpu-baseline --no-strong --no-post > "$OUT/${W}_ms.json" 2> "$OUT/${W}_ms.err" || { tail "$OUT/${W}_ms.err"; exit 1; }
  KMS=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['roofline']['kernel_ms_avg'])" "$OUT/${W}_ms.json")
  python3 tools/valu_profile.py "$OUT/sq_$W/summary.json" $W "$KMS" && cp profiles/valu_$W.json "$OUT/valu_$W.json"
done
bash tools/gpu_r03.sh "$TAG" evidence:aead:--no-strong evidence:encap
