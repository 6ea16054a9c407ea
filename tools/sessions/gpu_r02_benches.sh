#!/bin/bash
# Bench lines only (no tests) for the given workloads, each under its own
# limit; the first failure ends the script.
# usage: tools/sessions/gpu_r02_benches.sh TAG workload [workload...]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for w in "$@"; do
  echo "== bench $w"
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --workload "$w" > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  python3 -c "import json; d=json.load(open('$OUT/bench_$w.json')); r=d['roofline']; print(d['value'], d['unit'], r['frac'], r['kernel_ms_avg'], r['measured_read_peak'], r.get('frac_of_measured_read_peak'), (d.get('strong_scaling') or {}).get('value'))"
done
