#!/bin/bash
# PMC of tools/exp/store_granularity (one counter per pass, kernel trace only)
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/store_gran
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 ./tools/exp/store_granularity 20 > $OUT/times.jsonl
cat $OUT/times.jsonl
cd /tmp
for C in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_$C -o run -- $ROOT/tools/exp/store_granularity 3 > $OUT/pmc_$C.log 2>&1
done
python3 - <<'PY'
import csv, glob, statistics, collections, json
out = {}
for C in ("WRITE_SIZE", "FETCH_SIZE"):
    v = collections.defaultdict(list)
    for f in glob.glob(f"/root/repo/gpurun_out/store_gran/pmc_{C}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            v[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    for k, x in v.items():
        out.setdefault(k, {})[C + "_KiB_median"] = statistics.median(x)
for k, d in out.items():
    d["write_bytes_per_slot"] = d.get("WRITE_SIZE_KiB_median", 0) * 1024 / (1 << 22)
    d["fetch_x2_bytes_per_slot"] = d.get("FETCH_SIZE_KiB_median", 0) * 2048 / (1 << 22)
print(json.dumps(out, indent=1))
json.dump(out, open("/root/repo/gpurun_out/store_gran/pmc.json", "w"), indent=1)
PY
cd "$ROOT"
for W in 1 0; do
  WG_GRO_WIDE=$W bash tools/pmc_profile.sh $OUT/gro_wide$W --workload gro --steps 10 --settle-seconds 0.1 --no-strong > $OUT/gro_wide$W.log 2>&1
  python3 -c "import json; d=json.load(open('$OUT/gro_wide$W/pmc_gro.json')); g=d['gro_finalize']; print('gro_wide=$W', g['read_bytes_corrected']/4194304, g['write_bytes']/4194304)"
done
