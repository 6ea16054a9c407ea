#!/bin/bash
# rocprofv3 PMC counters of one bench.py workload's kernel, one pass per
# counter group (each group within the per-pass slot limits of
# MI355X_MICROARCH.md "rocprofv3 PMC slots"), kernel trace only.  Writes
# <outdir>/summary.json: the full kernel name(s) matching the substring and the
# per-dispatch median of every counter.
# usage: tools/counters.sh <outdir> <workload> <kernel-substring> "<pass 1 counters>" ["<pass 2>" ...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); W=$2; K=$3; shift 3
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$i" -o run -- \
     python3 "$ROOT/tools/verify_counter_run.py" "$W" > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($C) failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" "$K" "$W" <<'PY'
import csv, glob, json, sys, collections
out, key, wl = sys.argv[1], sys.argv[2], sys.argv[3]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {"workload": wl, "kernel_substring": key, "kernels": {}}
for k, cs in agg.items():
    res["kernels"][k] = {c: sorted(v)[len(v) // 2] for c, v in sorted(cs.items())}
    res["kernels"][k]["dispatches"] = max(len(v) for v in cs.values())
json.dump(res, open(out + "/summary.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
