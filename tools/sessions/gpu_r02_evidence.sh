#!/bin/bash
# Round-2 evidence session: GPU tests, host-path rates, bench lines for the
# given workloads (the first is profiled with rocprofv3 kernel stats, same
# box).  Every GPU step has its own limit; the first failure ends the script.
# usage: tools/sessions/gpu_r02_evidence.sh TAG workload [workload...]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
TAG=$1
shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
echo "== host path"
timeout -k 10 300 python3 tools/host_path.py > "$OUT/host_path.json" 2> "$OUT/host_path.err"
cat "$OUT/host_path.json"
for w in "$@"; do
  echo "== bench $w"
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --workload "$w" > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  python3 -c "import json; d=json.load(open('$OUT/bench_$w.json')); r=d['roofline']; print(d['value'], d['unit'], r['frac'], r['kernel_ms_avg'], r['measured_read_peak'], r.get('read_probe_variants'), (d.get('strong_scaling') or {}).get('value'))"
done
w=$1
echo "== rocprofv3 kernel stats: $w"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$w" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline --no-strong --workload "$w" > "$OUT/prof_$w.json" 2> "$OUT/prof_$w.err"
find "$OUT/prof_$w" -name "*kernel_stats.csv" -exec head -4 {} \;
echo done
