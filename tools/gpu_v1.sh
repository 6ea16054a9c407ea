set -o pipefail
T=${1:-v2}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_aead.py tests/test_gpu_hostpath.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.txt 2>&1 || { tail -30 gpurun_out/$T/pytest.txt; exit 1; }
tail -1 gpurun_out/$T/pytest.txt
for r in 1 2; do for v in 1 2; do
WG_AEAD_PAIR=$v timeout -k 10 300 python3 -u bench.py --workload aead --no-cpu-baseline --no-strong > gpurun_out/$T/aead_p$v.r$r.json 2> gpurun_out/$T/aead_p$v.err || exit 1
python3 -c "
import json,sys
d=json.loads(open('gpurun_out/$T/aead_p$v.r$r.json').read().strip().splitlines()[-1])
print('pair=$v', d['ms_per_step'], json.dumps(d['post_checks'].get('decap_fused')))"
done; done
