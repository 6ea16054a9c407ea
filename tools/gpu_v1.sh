set -o pipefail
T=${1:-v2}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_verify_gates.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.txt 2>&1 || { tail -30 gpurun_out/$T/pytest.txt; exit 1; }
tail -2 gpurun_out/$T/pytest.txt
timeout -k 10 400 python3 -u tools/verify_ab.py verify_small=0 verify_small=7 verify_small=6 > gpurun_out/$T/verify_ab.json 2>&1 || { tail -30 gpurun_out/$T/verify_ab.json; exit 1; }
tail -1 gpurun_out/$T/verify_ab.json | python3 -c "
import json,sys
d=json.load(sys.stdin)['verify_ab']
for b,v in d.items(): print(b, {k:(x['ms_med'],x['roofline_frac'],x['bit_exact_vs_first']) for k,x in v['variants'].items()})"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$T/prof -o run --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/verify_ab.py verify_small=6 --rounds 2 --batches 1500B,64B,c4mix,mix12 > $GRAFT_REPO_ROOT/gpurun_out/$T/prof_ab.txt 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/$T/prof -name "*kernel_stats.csv" -exec grep -i "verify" {} \; | cut -c1-200
