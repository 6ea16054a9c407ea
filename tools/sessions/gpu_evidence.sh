#!/bin/bash
# One GPU-box session: the whole -m gpu suite, smoke(), then per workload
# (config 2 = the metric's config, config 3 GSO, f1 verify, f2 GRO) the
# rocprofv3 kernel stats and the PMC HBM traffic (one counter per pass), the
# fresh PMC summary copied over the box's profiles/pmc_<w>.json so the bench
# lines that follow carry it, then the bench lines: the default run (config 2)
# and configs 3/4/5, verify, GRO.  Each GPU step has its own time limit; the
# first failure ends it.
# usage: tools/sessions/gpu_evidence.sh [outdir-name]
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-evidence}; mkdir -p $O
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
for W in config2 config3 verify gro; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/stats_$W" -o run --output-format csv -- python3 "$ROOT/bench.py" --workload $W --steps 30 --no-cpu-baseline > "$O/stats_$W.log" 2>&1) || { echo "stats $W failed"; tail "$O/stats_$W.log"; exit 1; }
  bash tools/pmc_profile.sh "$O/pmc_$W" --workload $W --steps 10 --settle-seconds 0.1 > "$O/pmc_$W.log" 2>&1 || { tail "$O/pmc_$W.log"; exit 1; }
  cp "$O/pmc_$W/pmc_$W.json" "profiles/pmc_$W.json"
  echo "profiled $W"
done
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
cat $O/bench_default.json
for W in config3 verify config5 config4 gro; do
  timeout -k 10 300 python3 bench.py --workload $W --steps 30 > $O/bench_$W.json 2> $O/bench_$W.err || { tail $O/bench_$W.err; exit 1; }
  cat $O/bench_$W.json
done
echo done
