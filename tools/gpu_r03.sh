#!/bin/bash
# Round-3 GPU session: the steps named on the command line, in order; every
# GPU step under its own time limit; the first failure ends the session.
#   tests              pytest -m gpu (whole suite)
#   verify_ab          tools/verify_ab.py (verify kernels on 1500-B / 64-B / mixed batches)
#   ab:W:V1:V2...      tools/ab.py W V1 V2 ...  (knob variants, e.g. ab:gro:gro_lds=1:gro_lds=2)
#   bench:W[:args]     python bench.py --workload W [args, comma-separated]
#   evidence:W[:args]  PMC passes of bench W (FETCH_SIZE, WRITE_SIZE) -> profiles/pmc_W.json on the
#                      box, THEN the bench line of W (its `traffic` is that PMC file), THEN the same
#                      bench under rocprofv3 --kernel-trace --stats (its per-dispatch average against
#                      the line's kernel_ms_isolated) — all on one box
#   n2                 bench.py --gpus 2 with gloo (two ranks on the one GPU)
#   abuild:NAME:W1,W2  tools/ab_builds.sh: tools/exp/variant_NAME/libwireglider_amd.so (A) against the
#                      tree's library (B), alternating processes, 3 rounds, on workloads W1, W2...
# usage: tools/gpu_r03.sh TAG step [step...]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=$1
shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fail() { echo "FAILED: $1"; [ -f "$2" ] && tail -25 "$2"; exit 1; }
for step in "$@"; do
  kind=${step%%:*}
  rest=${step#*:}
  echo "== $step  ($(date +%T))"
  case $kind in
    tests)
      timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$OUT/pytest_gpu.txt" 2>&1 || fail tests "$OUT/pytest_gpu.txt"
      tail -1 "$OUT/pytest_gpu.txt" ;;
    verify_ab)
      timeout -k 10 300 python3 -u tools/verify_ab.py > "$OUT/verify_ab.json" 2>&1 || fail verify_ab "$OUT/verify_ab.json"
      tail -1 "$OUT/verify_ab.json" | cut -c1-400 ;;
    ab)
      W=${rest%%:*}
      V=${rest#*:}
      timeout -k 10 300 python3 -u tools/ab.py "$W" ${V//:/ } > "$OUT/ab_$W.json" 2>&1 || fail "ab $W" "$OUT/ab_$W.json"
      cat "$OUT/ab_$W.json" ;;
    bench)
      W=${rest%%:*}
      A=""
      [ "$rest" != "$W" ] && A=${rest#*:}
      timeout -k 10 400 python3 -u bench.py --workload "$W" ${A//,/ } > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err" \
        || fail "bench $W" "$OUT/bench_$W.err"
      cut -c1-300 "$OUT/bench_$W.json" ;;
    evidence)
      W=${rest%%:*}
      A=""
      [ "$rest" != "$W" ] && A=${rest#*:}
      bash tools/pmc_profile.sh "$OUT/pmc_$W" --workload "$W" --steps 10 --settle-seconds 0.1 --no-strong \
        > "$OUT/pmc_$W.log" 2>&1 || fail "pmc $W" "$OUT/pmc_$W.log"
      cp "$OUT/pmc_$W/pmc_$W.json" "$ROOT/profiles/pmc_$W.json"
      timeout -k 10 500 python3 -u bench.py --workload "$W" ${A//,/ } > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err" \
        || fail "evidence bench $W" "$OUT/bench_$W.err"
      cut -c1-300 "$OUT/bench_$W.json"
      (cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$W" -o run --output-format csv -- \
        python3 -u "$ROOT/bench.py" --workload "$W" --no-cpu-baseline --no-post --no-strong > "$OUT/stats_bench_$W.json" \
        2> "$OUT/stats_bench_$W.err") || fail "evidence stats $W" "$OUT/stats_bench_$W.err"
      find "$OUT/stats_$W" -name "*kernel_stats.csv" -exec head -4 {} \; ;;
    abuild)
      N=${rest%%:*}
      W=${rest#*:}
      timeout -k 10 900 bash tools/ab_builds.sh "$OUT/abuild_$N.jsonl" 3 "tools/exp/variant_$N/libwireglider_amd.so" \
        "$ROOT/wireglider_amd/lib/libwireglider_amd.so" ${W//,/ } > "$OUT/abuild_$N.txt" 2>&1 || fail "abuild $N" "$OUT/abuild_$N.txt"
      cat "$OUT/abuild_$N.txt" ;;
    n2)
      WG_DIST_BACKEND=gloo timeout -k 10 500 python3 -u bench.py --gpus 2 --steps 10 --no-cpu-baseline \
        > "$OUT/bench_n2.json" 2> "$OUT/bench_n2.err" || fail n2 "$OUT/bench_n2.err"
      cut -c1-300 "$OUT/bench_n2.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session $TAG done ($(date +%T))"
