set -o pipefail
T=${1:-v2}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_verify_gates.py tests/test_gpu_l4.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.txt 2>&1 || { tail -30 gpurun_out/$T/pytest.txt; exit 1; }
tail -2 gpurun_out/$T/pytest.txt
timeout -k 10 400 python3 -u tools/verify_ab.py verify_small=7 verify_small=7,verify_stage=0 --batches 64B,alt,mix25,c4mix,1500B > gpurun_out/$T/verify_ab.json 2>&1 || { tail -30 gpurun_out/$T/verify_ab.json; exit 1; }
tail -1 gpurun_out/$T/verify_ab.json | python3 -c "
import json,sys
d=json.load(sys.stdin)['verify_ab']
for b,v in d.items(): print(b, {k:(x['ms_med'],x['roofline_frac'],x['bit_exact_vs_first']) for k,x in v['variants'].items()})"
for W in verify64:verify_stage config4small:l4_stage config4:l4_stage config5:l4_stage; do
  w=${W%%:*}; k=${W#*:}
  timeout -k 10 300 python3 -u tools/ab.py $w $k=1 $k=0 > gpurun_out/$T/ab_$w.json 2>&1 || { tail -30 gpurun_out/$T/ab_$w.json; exit 1; }
  tail -1 gpurun_out/$T/ab_$w.json
done
