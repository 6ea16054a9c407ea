#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r02f; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_verify_gates.py tests/test_gpu_l4.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 tools/ab.py verify verify_small=0 verify_small=3 verify_small=1 > $OUT/ab_verify.json; cat $OUT/ab_verify.json
timeout -k 10 400 python3 bench.py --workload verify --steps 20 --warmup 3 --no-strong --no-cpu-baseline > $OUT/bench_verify.json
python3 -c "
import json; d=json.load(open('$OUT/bench_verify.json'))
print(json.dumps({k: (v['kernel_ms'] if isinstance(v, dict) else v) for k, v in d['post_checks']['small_64B'].items()}))"
