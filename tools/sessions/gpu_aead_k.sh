#!/bin/bash
# SQ counters of the AEAD kernel at aead_k = 1, 2, 4 (one --pmc pass each,
# kernel trace only), on the bench.py aead workload.
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/aead_k
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for K in 1 2 4; do
  WG_AEAD_K=$K timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace \
    --output-format csv -d $OUT/k$K -o run -- python3 $ROOT/bench.py --workload aead --steps 5 --warmup 1 --settle-seconds 0.05 \
    --no-strong --no-cpu-baseline > $OUT/k$K.log 2>&1
done
python3 - <<'PY'
import csv, glob, statistics, collections, json
out = {}
for K in (1, 2, 4):
    v = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"/root/repo/gpurun_out/aead_k/k{K}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "aead_kernel" in r["Kernel_Name"]:
                v[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out[K] = {k: {c: statistics.median(x) for c, x in d.items()} for k, d in v.items()}
print(json.dumps(out, indent=1))
json.dump(out, open("/root/repo/gpurun_out/aead_k/pmc.json", "w"), indent=1)
PY
