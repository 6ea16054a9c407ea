#!/bin/bash
# Round 6: the simplified verify state (handle keys, per-thread serial for
# hipStreamPerThread, no events) — MT + verify suites, launch rates (full and
# small batches, 1 / 4 / 16 threads), and the first-call verify kernel under
# rocprofv3.
set -u
O=gpurun_out/r6d; mkdir -p $O
ok() { local rc=$1; if [ "$rc" -ge 124 ]; then echo "stop: rc $rc"; exit "$rc"; fi; }
timeout -k 10 900 python3 -u -m pytest tests/test_mt_batch.py tests/test_verify_gates.py -x -v -s -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_mt_verify.txt 2>&1; rc=$?; grep -E "passed|failed" $O/pytest_mt_verify.txt | tail -3; ok $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "
import sys; sys.path[:0] = ['tests', 'oracle']
from pathlib import Path
import test_mt_batch as t
d = Path('$O/mt_in'); d.mkdir(exist_ok=True); t.write_inputs(d)"; ok $?
for B in full small; do
  for T in 1 4 16; do
    timeout -k 10 200 tests/cpp/bin/mt_batch $O/mt_in rate $T 2000 $B > $O/rate_${B}_$T.json 2>$O/rate_${B}_$T.err; rc=$?
    echo "rate $B $T rc $rc"; ok $rc
  done
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fc -o fc -- python3 tools/verify_first_call.py > $O/first_call.json 2>$O/first_call.err; rc=$?
echo "first call rc $rc: $(cat $O/first_call.json)"; ok $rc
rm -rf $O/mt_in
