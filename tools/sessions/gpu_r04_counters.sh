#!/bin/bash
# Round 4, first call: PMC counters of the kernels VERDICT r03 names
# (config 4's 64-B sub-batch, the AEAD encrypt, the verify lane kernel) and of
# config 2's kernel for comparison.  usage: tools/sessions/gpu_r04_counters.sh TAG
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM"
SQ2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR"
TA="TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT"
TC="TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum"
run() { echo "== $*  ($(date +%T))"; bash tools/counters.sh "$@" > "$OUT/$(basename "$1").log" 2>&1 || { tail -20 "$OUT/$(basename "$1").log"; exit 1; }; }
run "$OUT/c4small" config4small l4csum_split_kernel "$SQ1" "$SQ2" "$TA" "$TC"
run "$OUT/config2" config2 l4csum_kernel "$SQ1" "$SQ2" "$TA" "$TC"
run "$OUT/aead" aead aead_kernel "$SQ1" "$SQ2"
run "$OUT/verify64d" verify64d verify_compact "$SQ1" "$SQ2" "$TA"
echo "session $TAG done ($(date +%T))"
