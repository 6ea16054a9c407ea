set -o pipefail
mkdir -p gpurun_out/sh8
export TMPDIR=/tmp
for r in 1 2; do for L in tools/exp/variant_sh8/libwireglider_amd.so wireglider_amd/lib/libwireglider_amd.so; do
  WG_LIB=$L timeout -k 10 300 python3 -u tools/verify_ab.py verify_small=6 verify_small=0 --batches 1500B,alt,mix25,c4mix --rounds 3 > gpurun_out/sh8/ab_$r.$(basename $(dirname $L)).json 2>&1 || { tail -20 gpurun_out/sh8/ab_$r.$(basename $(dirname $L)).json; exit 1; }
  echo "$L"; tail -1 gpurun_out/sh8/ab_$r.$(basename $(dirname $L)).json | python3 -c "
import json,sys
d=json.load(sys.stdin)['verify_ab']
for b,v in d.items(): print(' ', b, {k:(x['ms_med'],x['bit_exact_vs_first']) for k,x in v['variants'].items()})"
done; done
