#!/bin/bash
# Round 6: the multi-thread suite with seven entry points and its launch
# rates on small batches (1 / 4 / 16 threads).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_mt_batch.py -v -s -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest_mt.txt 2>&1 || { tail -30 $O/pytest_mt.txt; exit 1; }
grep -E "passed|failed" $O/pytest_mt.txt | tail -2
timeout -k 10 300 python3 -c "
import sys; sys.path[:0] = ['tests', 'oracle']
from pathlib import Path
import test_mt_batch as t
d = Path('$O/mt_in'); d.mkdir(exist_ok=True); t.write_inputs(d)" || exit 1
for T in 1 4 16; do
  timeout -k 10 200 tests/cpp/bin/mt_batch $O/mt_in rate $T 500 small > $O/rate_small_$T.json 2> $O/rate_small_$T.err || exit 1
  echo "rate $T done"
done
rm -rf $O/mt_in
