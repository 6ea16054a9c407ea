#!/bin/bash
# SQ instruction / wait counters of one bench.py workload's kernels, two
# passes of 8 SQ counters; per-kernel medians per launch in summary.txt.
# usage: tools/kernel_counters.sh <outdir> <workload> <kernel-name-substring>
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); W=$2; K=$3; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM"
P2="SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_RD"
i=0
for C in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$i" -o run -- \
     python3 "$ROOT/tools/verify_counter_run.py" "$W" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" "$K" > "$OUT/summary.txt" <<'PY'
import csv, glob, sys, collections
out, key = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(key, {c: round(sorted(v)[len(v)//2], 1) for c, v in sorted(agg.items())})
PY
cat "$OUT/summary.txt"
