#!/bin/bash
# HBM traffic of the bench kernel from rocprofv3 PMC counters, one counter per
# pass (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950), kernel
# trace only — no sys/runtime trace alongside --pmc.
# usage: tools/pmc_profile.sh <outdir> [bench args...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o run -- \
      python3 "$ROOT/bench.py" --no-cpu-baseline --no-post "$@" > "$OUT/pmc_$C.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "rocprofv3 --pmc $C failed rc=$rc"; tail -20 "$OUT/pmc_$C.log"; exit $rc; fi
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT" "$@"
