#!/bin/bash
# Round 4 encap synthesis: where the time goes — rocprofv3 kernel statistics
# of the encap step with encap_synth 0 / 1, SQ counters of the synthesizing
# AEAD kernel.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for S in 0 1; do
  (cd /tmp && WG_ENCAP_SYNTH=$S timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_synth$S" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --workload encap --steps 10 --no-cpu-baseline --no-strong --no-post > "$OUT/stats_synth$S.log" 2>&1) || { echo "stats $S failed"; tail "$OUT/stats_synth$S.log"; exit 1; }
  python3 - "$OUT/stats_synth$S" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{float(r['AverageNs'])/1e3:10.1f} us x {r['Calls']:>5}  {r['Name'][:110]}")
PY
done
WG_ENCAP_SYNTH=1 timeout -k 10 400 bash tools/counters.sh "$OUT/sq1" encap aead_kernel \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
  "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH" > "$OUT/sq1.log" 2>&1 || { tail -20 "$OUT/sq1.log"; exit 1; }
WG_ENCAP_SYNTH=0 timeout -k 10 400 bash tools/counters.sh "$OUT/sq0" encap aead_kernel \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" > "$OUT/sq0.log" 2>&1 || { tail -20 "$OUT/sq0.log"; exit 1; }
cat "$OUT/sq1/summary.json" "$OUT/sq0/summary.json"
echo "session $TAG done"
