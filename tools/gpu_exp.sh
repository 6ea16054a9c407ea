set -o pipefail
mkdir -p gpurun_out/v5
B=1500B,64B,c4mix,mix25
for k in 0 1 2; do
WG_EXPD64=1 WG_EXPK2=$k timeout -k 10 200 python3 -u tools/verify_ab.py verify_small=0 verify_small=7 verify_small=6 --batches $B --rounds 4 > gpurun_out/v5/ab_k$k.json 2>&1 || exit 1
echo k$k; tail -1 gpurun_out/v5/ab_k$k.json | python3 -c "
import json,sys
d=json.load(sys.stdin)['verify_ab']
for b,v in d.items(): print(b, {k:(x['ms_med'],x['bit_exact_vs_first']) for k,x in v['variants'].items()})"
done
