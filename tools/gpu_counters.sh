#!/bin/bash
# One rocprofv3 --pmc pass (kernel trace only) per counter set over a
# bench.py workload; medians per kernel and counter into
# gpurun_out/counters/<tag>/summary.json.
# usage: tools/gpu_counters.sh TAG WORKLOAD "C1 C2 ..." ["C1 C2 ..." ...]
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
ROOT=$(pwd)
TAG=$1
W=$2
shift 2
OUT=$ROOT/gpurun_out/counters/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for set in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python3 $ROOT/bench.py --workload $W --steps 5 --warmup 1 --settle-seconds 0.05 --no-strong --no-cpu-baseline \
    > $OUT/p$i.log 2>&1
  i=$((i + 1))
done
python3 - "$OUT" <<'PY'
import csv, glob, statistics, collections, json, sys
out = sys.argv[1]
v = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        v[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: {c: statistics.median(x) for c, x in d.items()} for k, d in v.items() if "probe" not in k and "synth" not in k}
print(json.dumps(res, indent=1))
json.dump(res, open(f"{out}/summary.json", "w"), indent=1)
PY
