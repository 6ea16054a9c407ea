#!/bin/bash
# Round 6: stream identity, the multi-thread harness before (round-5 verify
# state, keyed by handle) and after the fix, the GPU verify / MT suites, and
# the launch-rate figure.  Every GPU step has its own time limit; a crash,
# abort or timeout ends the script.
set -u
O=gpurun_out/r6b; mkdir -p $O
ok() { local rc=$1; if [ "$rc" -ge 124 ]; then echo "stop: rc $rc"; exit "$rc"; fi; }
timeout -k 10 120 ./tools/exp/bin/stream_identity > $O/stream_identity.txt 2>&1; ok $?
cat $O/stream_identity.txt
timeout -k 10 300 python3 -c "
import sys; sys.path[:0] = ['tests', 'oracle']
from pathlib import Path
import test_mt_batch as t
d = Path('$O/mt_in'); d.mkdir(exist_ok=True); print(t.write_inputs(d))" > $O/inputs.txt 2>&1; ok $?
for vs in 6 7; do
  for mode in perthread churn own; do
    WG_VERIFY_SMALL=$vs LD_LIBRARY_PATH=$PWD/tools/exp/variant_r05verify timeout -k 10 120 \
      tests/cpp/bin/mt_batch $O/mt_in conform 4 50 $mode > $O/before_${mode}_vs$vs.json 2>$O/before_${mode}_vs$vs.err
    rc=$?; echo "before $mode vs$vs rc $rc: $(cat $O/before_${mode}_vs$vs.json)"; ok $rc
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_mt_batch.py tests/test_verify_gates.py -x -v -s -m gpu \
  --timeout 200 --timeout-method thread > $O/pytest_mt_verify.txt 2>&1; rc=$?; tail -5 $O/pytest_mt_verify.txt; ok $rc
for T in 1 4 16; do
  timeout -k 10 200 tests/cpp/bin/mt_batch $O/mt_in rate $T 2000 > $O/rate_$T.json 2>$O/rate_$T.err; rc=$?
  echo "rate $T rc $rc: $(cat $O/rate_$T.json)"; ok $rc
done
