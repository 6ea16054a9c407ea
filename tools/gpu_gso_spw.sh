#!/bin/bash
# GSO parity under every split variant (incl. the S = 3 / 4 segment batches)
# and the config 3 / fused encap bench lines.  usage: tools/gpu_gso_spw.sh TAG
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gso.py tests/test_gpu_encap.py > "$OUT/pytest.log" 2>&1
tail -1 "$OUT/pytest.log"
for w in config3 encap; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --workload $w --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  python3 -c "import json; d=json.load(open('$OUT/bench_$w.json')); r=d['roofline']; print('$w', d['value'], d['ms_per_step'], r['frac'], r.get('frac_of_measured_read_peak'))"
done
