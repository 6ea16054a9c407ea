#!/bin/bash
# SQ counters of the GSO split kernel at gso_groups G (env WG_GSO_GROUPS),
# two passes of 8 SQ counters each; per-launch medians in summary_G<G>.txt.
# usage: tools/gso_counters2.sh <outdir> <G>...
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM"
P2="SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR"
for G in "$@"; do
  i=0; mkdir -p "$OUT/g$G"
  for C in "$P1" "$P2"; do
    i=$((i+1))
    WG_GSO_GROUPS=$G timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/g$G/p$i" -o run -- \
       python3 "$ROOT/tools/gso_counter_run.py" > "$OUT/g$G/p$i.log" 2>&1 || { echo "G=$G pass $i failed"; tail -5 "$OUT/g$G/p$i.log"; exit 1; }
  done
  python3 - "$OUT/g$G" > "$OUT/summary_G$G.txt" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        k = "split" if "gso_split_kernel" in k else "copy" if "probe_copy" in k else None
        if k: agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sorted(v)[len(v)//2], 1) for c, v in sorted(d.items())})
PY
  cat "$OUT/summary_G$G.txt"
done
