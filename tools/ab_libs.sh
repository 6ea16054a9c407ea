#!/bin/bash
# Same-box A/B of N library builds: alternating processes, one bench line
# each (kernel ms), R rounds.
# usage: tools/ab_libs.sh <out.jsonl> <R> <workload[,workload...]> <lib>...
set -u
OUT=$1; R=$2; WS=$3; shift 3
: > "$OUT"
# each library's GPU parity subset first (AB_GSO=1: + the GSO suite); the
# timing rows follow, and the summary names every library's parity
for L in "$@"; do
  tools/ab_parity.sh "$OUT" "$L" ${AB_GSO:+gso} || exit 1
done
for r in $(seq "$R"); do
  for W in ${WS//,/ }; do
    for L in "$@"; do
      WG_LIB=$L timeout -k 10 300 python3 bench.py --workload "$W" --steps 30 --no-cpu-baseline --no-strong --no-post 2>>"$OUT.err" | \
        python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': sys.argv[1], 'workload': sys.argv[2], 'kernel_ms': d['roofline'].get('kernel_ms_avg', d['ms_per_step'])}))" "$L" "$W" >> "$OUT" || exit 1
    done
  done
done
python3 - "$OUT" <<'PY'
import json, sys, statistics, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
par = {r["lib"]: r["parity"] for r in rows if "parity" in r}
rows = [r for r in rows if "kernel_ms" in r]
g = collections.defaultdict(list)
for r in rows: g[(r["workload"], r["lib"])].append(r["kernel_ms"])
for (w, l), v in sorted(g.items()): print(w, l, "parity", par.get(l, "not run"), "median ms", round(statistics.median(v), 5), "all", v)
PY
