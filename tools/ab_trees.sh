#!/bin/bash
# Same-box A/B of two source trees' bench.py (each with its own in-tree
# library): alternating processes, one line each (kernel ms), R rounds.
# Used for round-3-final vs current: the C ABI changed in
# between, so each tree runs its own Python binding and bench.
# usage: tools/ab_trees.sh <out.jsonl> <R> <workload[,workload...]> <treeA> <treeB>
set -u
OUT=$1; R=$2; WS=$3; A=$4; B=$5
: > "$OUT"
HERE=$(pwd); OUTABS=$(realpath -m "$OUT")
# each tree's GPU parity subset first, run in that tree against its own
# library (AB_GSO=1: + GSO)
for T in "$A" "$B"; do
  (cd "$T" && "$HERE"/tools/ab_parity.sh "$OUTABS" "$(realpath "$T")/wireglider_amd/lib/libwireglider_amd.so" \
     ${AB_GSO:+gso}) || exit 1
done
for r in $(seq "$R"); do
  for W in ${WS//,/ }; do
    for T in "$A" "$B"; do
      (cd "$T" && timeout -k 10 300 python3 bench.py --workload "$W" --steps 30 --no-cpu-baseline --no-strong --no-post) 2>>"$OUT.err" | \
        python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'tree': sys.argv[1], 'workload': sys.argv[2], 'kernel_ms': d['roofline']['kernel_ms_avg'], 'frac': d['roofline']['frac']}))" "$T" "$W" >> "$OUT" || exit 1
    done
  done
done
python3 - "$OUT" <<'PY'
import json, os, sys, statistics, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
par = {r["lib"].rsplit("/wireglider_amd/lib/", 1)[0]: r["parity"] for r in rows if "parity" in r}
rows = [r for r in rows if "kernel_ms" in r]
g = collections.defaultdict(list)
for r in rows: g[(r["workload"], r["tree"])].append(r["kernel_ms"])
for (w, t), v in sorted(g.items()): print(w, t, "parity", par.get(os.path.realpath(t), "not run"), "median ms", round(statistics.median(v), 5), "all", v)
PY
