#!/bin/bash
# Round 4: SQ counters of the timed AEAD kernel (the staged-message build) for
# profiles/valu_aead.json, then bench lines whose CPU baselines showed the
# widest spreads, with the quiet-CPU pinning.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 bash tools/counters.sh "$OUT/sq" aead aead_kernel \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
  "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH" \
  "GRBM_GUI_ACTIVE GRBM_COUNT" > "$OUT/sq.log" 2>&1 || { tail -20 "$OUT/sq.log"; exit 1; }
bash tools/gpu_r03.sh "$TAG" bench:aead:--no-strong bench:config2 bench:config5:--no-strong bench:config3udp bench:verify:--no-strong bench:encap
