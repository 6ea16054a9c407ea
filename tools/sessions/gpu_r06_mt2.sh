#!/bin/bash
# Round 6 (after the fix): stream semantics on both HIP runtimes of the
# image (ROCm 7.2 in /opt/rocm, PyTorch's bundled 7.0), the multi-thread
# harness suite and the verify suite against the fixed library, and the
# launch-rate figure.  Each GPU step has its own limit; a crash, abort or
# timeout ends the script.
set -u
O=gpurun_out/r6c; mkdir -p $O
ok() { local rc=$1; if [ "$rc" -ge 124 ]; then echo "stop: rc $rc"; exit "$rc"; fi; }
TL=$(python3 -c "import os, torch; print(os.path.dirname(torch.__file__) + '/lib')")
mkdir -p /tmp/rt70 && ln -sf "$TL/libamdhip64.so" /tmp/rt70/libamdhip64.so.7
timeout -k 10 120 ./tools/exp/bin/stream_identity > $O/stream_identity_rocm72.txt 2>&1; ok $?
LD_LIBRARY_PATH=/tmp/rt70:$TL timeout -k 10 120 ./tools/exp/bin/stream_identity_nogetid > $O/stream_identity_torch70.txt 2>&1; ok $?
head -20 $O/stream_identity_rocm72.txt; head -20 $O/stream_identity_torch70.txt
timeout -k 10 900 python3 -u -m pytest tests/test_mt_batch.py tests/test_verify_gates.py -x -v -s -m gpu \
  --timeout 300 --timeout-method thread > $O/pytest_mt_verify.txt 2>&1; rc=$?; grep -E "passed|failed|mismatched" $O/pytest_mt_verify.txt | tail -25; ok $rc
[ $rc -eq 0 ] || exit $rc
D=$(ls -d /tmp/pytest-of-*/pytest-*/mt_batch0 2>/dev/null | head -1)
[ -n "$D" ] || { python3 -c "
import sys; sys.path[:0] = ['tests', 'oracle']
from pathlib import Path
import test_mt_batch as t
d = Path('$O/mt_in'); d.mkdir(exist_ok=True); t.write_inputs(d)"; D=$O/mt_in; }
for T in 1 4 16; do
  timeout -k 10 200 tests/cpp/bin/mt_batch $D rate $T 2000 > $O/rate_$T.json 2>$O/rate_$T.err; rc=$?
  echo "rate $T rc $rc: $(cat $O/rate_$T.json)"; ok $rc
done
