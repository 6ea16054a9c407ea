#!/bin/bash
# Host-path step time per host_chunk_mb, one process per point (a copy-engine
# pathology can stick to a process): encap_host and decap_host.
# usage: tools/host_chunk_sweep.sh <out.jsonl> [MiB ...]
set -u
OUT=$1; shift
: > "$OUT"
for W in encap_host decap_host; do
  for MB in "${@:-16 32 64 128 256}"; do
    WG_HOST_CHUNK_MB=$MB timeout -k 10 300 python3 bench.py --workload $W --steps 10 --no-cpu-baseline --no-post --no-strong \
      2>>"$OUT.err" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'workload': sys.argv[1], 'host_chunk_mb': int(sys.argv[2]), 'ms_per_step': d['ms_per_step'], 'frac_of_pcie_both': d['roofline']['frac']}))" $W $MB >> "$OUT" || exit 1
  done
done
cat "$OUT"
