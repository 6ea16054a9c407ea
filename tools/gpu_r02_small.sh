set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r02c; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_l4.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_l4.log 2>&1 || { tail -30 $OUT/pytest_l4.log; exit 1; }
tail -1 $OUT/pytest_l4.log
timeout -k 10 300 python3 tools/ab.py config5 l4_small=0 l4_small=5 l4_small=2 > $OUT/ab_config5.json; cat $OUT/ab_config5.json
timeout -k 10 300 python3 tools/ab.py config4 l4_small=0 l4_small=5 > $OUT/ab_config4.json; cat $OUT/ab_config4.json
timeout -k 10 400 python3 bench.py --workload config4 --steps 20 --warmup 3 --no-strong --no-cpu-baseline > $OUT/bench_config4.json; python3 -c "
import json; d=json.load(open('$OUT/bench_config4.json'))
for k,v in d['post_checks']['sub_batches'].items(): print(k, json.dumps(v))"
