#!/bin/bash
# rocprofv3 kernel stats + PMC HBM traffic for the SURVEY §8 f-row workloads
# (verify = f1 wg_verify_desc, gro = f2 wg_gro_finalize).  Each GPU step has
# its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
O=$ROOT/gpurun_out/frows_prof; mkdir -p "$O"
WL=${@:-verify gro}
export TMPDIR=/tmp
for W in $WL; do
  timeout -k 10 300 python3 bench.py --workload $W --steps 100 > "$O/bench_$W.json" 2> "$O/bench_$W.err" || { tail "$O/bench_$W.err"; exit 1; }
  cat "$O/bench_$W.json"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/stats_$W" -o run --output-format csv -- python3 "$ROOT/bench.py" --workload $W --steps 100 --no-cpu-baseline > "$O/stats_$W.log" 2>&1) || { echo "stats $W failed"; exit 1; }
  bash tools/pmc_profile.sh "$O/pmc_$W" --workload $W --steps 20 > "$O/pmc_$W.log" 2>&1 || { tail "$O/pmc_$W.log"; exit 1; }
done
echo done
