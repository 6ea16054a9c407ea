#!/bin/bash
# Round 4: rocprofv3 kernel statistics of the encap step and the aead line
# (which kernels, how long each).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for W in ${2:-encap aead}; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$W" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --workload $W --steps 20 --no-cpu-baseline --no-strong --no-post > "$OUT/stats_$W.log" 2>&1) || { echo "stats $W failed"; tail "$OUT/stats_$W.log"; exit 1; }
  python3 - "$OUT/stats_$W" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{float(r['AverageNs'])/1e3:10.1f} us x {r['Calls']:>5}  {r['Name'][:110]}")
PY
done
echo "session $TAG done"
