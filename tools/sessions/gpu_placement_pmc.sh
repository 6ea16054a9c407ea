#!/bin/bash
# Address-translation counters of the config 5 kernel per allocation
# (tools/placement_probe.py, 5 allocations, 3 launches each, one --pmc pass
# with kernel trace only).
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/place_pmc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
PROBE_K=3 PROBE_SETTLE=0 timeout -s KILL 240 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
  TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_PERMISSION_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d $OUT/pmc -o run -- python3 $ROOT/tools/placement_probe.py config5 5 > $OUT/pmc.log 2>&1
python3 - <<'PY'
import csv, glob, json, collections
rows = []
for f in glob.glob("/root/repo/gpurun_out/place_pmc/pmc/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
by = collections.OrderedDict()
for r in rows:
    key = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
    d = by.setdefault(key, {"kernel": r["Kernel_Name"]})
    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
seq = [dict(id=k, **v) for k, v in sorted(by.items()) if "l4csum" in v["kernel"]]
groups, cur, last = [], [], None
for d in seq:
    if last is not None and d["id"] != last + 1:
        groups.append(cur); cur = []
    cur.append(d); last = d["id"]
groups.append(cur)
out = []
for g in groups:
    m = {c: sorted(x[c] for x in g)[len(g) // 2] for c in g[0] if c not in ("kernel", "id")}
    out.append({"dispatches": [x["id"] for x in g], **m})
print(json.dumps(out, indent=1))
json.dump(out, open("/root/repo/gpurun_out/place_pmc/summary.json", "w"), indent=1)
PY
grep '"alloc"' $OUT/pmc.log | head -20
