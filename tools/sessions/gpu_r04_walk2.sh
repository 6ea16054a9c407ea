#!/bin/bash
# Round 4: the walking verify kernel with two descriptors per lane (72 VGPRs,
# 7 waves per SIMD as before, half the waves) — verify parity, then
# alternating-process A/B against one descriptor per lane
# (tools/exp/variant_walk1), and the first call on fresh streams.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_verify_gates.py tests/test_gpu_golden_l4.py tests/test_gpu_hostpath.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
timeout -k 10 900 bash tools/ab_libs.sh "$OUT/ab.jsonl" 3 verify64d,verify,config4 wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_walk1/libwireglider_amd.so > "$OUT/ab.txt" 2>&1 || { tail "$OUT/ab.txt"; tail "$OUT/ab.jsonl.err"; exit 1; }
cat "$OUT/ab.txt"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/first" -o run --output-format csv -- \
  python3 "$ROOT/tools/verify_first_call.py" > "$OUT/first.log" 2>&1) || { echo "first-call run failed"; tail "$OUT/first.log"; exit 1; }
python3 - "$OUT/first" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{float(r['AverageNs'])/1e3:10.2f} us x {r['Calls']:>5}  {r['Name'][:90]}")
PY
echo "session $TAG done"
