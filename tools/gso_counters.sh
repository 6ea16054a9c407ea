#!/bin/bash
# Counter study of the GSO kernel vs the copy probe (one counter group per pass).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
CGROUPS=${GSO_COUNTER_GROUPS:-"SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY|TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum|TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum|TCC_HIT_sum TCC_MISS_sum|TA_BUSY_avr TD_BUSY_avr"}
IFS='|' read -r -a GARR <<< "$CGROUPS"
for C in "${GARR[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$i" -o run -- \
     python3 "$ROOT/tools/gso_counter_run.py" > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($C) failed"; tail -5 "$OUT/p$i.log"; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        k = ("gso" if "gso_split_kernel" in k else "seg" if "gso_seg_kernel" in k
             else "plan" if "gso_plan_kernel" in k else ("copy" if "probe_copy" in k else None))
        if k: agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sorted(v)[len(v)//2], 1) for c, v in sorted(d.items())})
PY
