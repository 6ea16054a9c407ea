#!/bin/bash
# Whole -m gpu suite, bench lines for config2 / config5 / verify, SQ counters
# of the verify and config5 kernels.
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-l4_check}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for W in config2 config5 verify; do
  timeout -k 10 300 python3 bench.py --workload $W --steps 30 --no-cpu-baseline > $O/bench_$W.json 2> $O/bench_$W.err || { tail $O/bench_$W.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms_avg'])" $O/bench_$W.json $W
done
bash tools/kernel_counters.sh $O/vctr verify verify_kernel && bash tools/kernel_counters.sh $O/c5ctr config5 l4csum_kernel
