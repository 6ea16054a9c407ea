#!/bin/bash
# Round 4 final evidence, part A: smoke, the whole GPU suite, SQ counters of
# the timed AEAD kernel (profiles/valu_aead.json, its symbol now carrying the
# synthesis flag), then PMC + line + kernel statistics for the AEAD, encap
# and config 2 lines, all on one box.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
bash tools/gpu_r03.sh "$TAG" tests || exit 1
timeout -k 10 400 bash tools/counters.sh "$OUT/sq_aead" aead aead_kernel \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
  "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH" \
  "GRBM_GUI_ACTIVE GRBM_COUNT" > "$OUT/sq_aead.log" 2>&1 || { tail -20 "$OUT/sq_aead.log"; exit 1; }
timeout -k 10 300 python3 -u bench.py --workload aead --steps 30 --no-cpu-baseline --no-strong --no-post > "$OUT/aead_ms.json" 2> "$OUT/aead_ms.err" || { tail "$OUT/aead_ms.err"; exit 1; }
KMS=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['roofline']['kernel_ms_avg'])" "$OUT/aead_ms.json")
python3 tools/valu_profile.py "$OUT/sq_aead/summary.json" aead "$KMS" && cp profiles/valu_aead.json "$OUT/valu_aead.json"
bash tools/gpu_r03.sh "$TAG" evidence:aead:--no-strong evidence:encap evidence:config2
