#!/bin/bash
# SQ instruction counters + kernel stats of the f4 AEAD kernels (one --pmc pass
# with kernel trace only), on the bench.py aead workload.
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/aead_pmc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d $OUT/pmc -o run -- python3 $ROOT/bench.py --workload aead --steps 5 --warmup 1 --settle-seconds 0.05 \
  --no-strong --no-cpu-baseline > $OUT/pmc.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/bench.py \
  --workload aead --steps 20 --warmup 3 --no-strong --no-cpu-baseline > $OUT/prof.log 2>&1
python3 - <<'PY'
import csv, glob, statistics, collections, json
v = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("/root/repo/gpurun_out/aead_pmc/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "aead_kernel" in r["Kernel_Name"]:
            v[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: statistics.median(x) for c, x in d.items()} for k, d in v.items()}
print(json.dumps(out, indent=1))
json.dump(out, open("/root/repo/gpurun_out/aead_pmc/pmc.json", "w"), indent=1)
PY
find $OUT/prof -name "*kernel_stats.csv" -exec head -4 {} \;
python3 - <<'PY'
import json
d = json.load(open("/root/repo/gpurun_out/aead_pmc/pmc.json"))
k = next(k for k in d if "aead_kernel" in k and "false" in k)
json.dump({"kernel": k, "valu_winst_per_launch": d[k]["SQ_INSTS_VALU"], "salu_winst_per_launch": d[k]["SQ_INSTS_SALU"],
           "waves": d[k]["SQ_WAVES"], "workload": "aead"}, open("/root/repo/gpurun_out/aead_pmc/valu_aead.json", "w"), indent=1)
PY
