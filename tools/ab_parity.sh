#!/bin/bash
# The GPU parity subset run against one library build (VERDICT r05 item 4:
# an A/B of a variant records the variant's parity, not only its timing).
# Appends one JSON line {"lib", "parity": "pass"|"fail", "tests", "summary"}
# to <out>.  usage: tools/ab_parity.sh <out.jsonl> <lib> [gso]
#   default subset: tests/test_gpu_l4.py tests/test_gpu_golden_l4.py
#   third argument "gso": + tests/test_gpu_gso.py; AB_PARITY_TESTS overrides.
set -u
OUT=$1; L=$2; KIND=${3:-}
TESTS=${AB_PARITY_TESTS:-"tests/test_gpu_l4.py tests/test_gpu_golden_l4.py"}
[ "$KIND" = gso ] && [ -z "${AB_PARITY_TESTS:-}" ] && TESTS="$TESTS tests/test_gpu_gso.py"
LOG=$(mktemp)
# shellcheck disable=SC2086
# WG_LIB for the Python binding; LD_LIBRARY_PATH for the C++ harnesses
# (tests/cpp/bin/*: their RUNPATH comes after it)
WG_LIB=$L LD_LIBRARY_PATH="$(dirname "$(realpath "$L")")${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH}" \
  timeout -k 10 900 python3 -m pytest $TESTS -q -m gpu --timeout 120 --timeout-method thread >"$LOG" 2>&1
RC=$?
python3 - "$OUT" "$L" "$RC" "$TESTS" "$LOG" <<'PY'
import json, sys
out, lib, rc, tests, log = sys.argv[1:6]
lines = [l for l in open(log).read().splitlines() if l.strip()]
summary = lines[-1] if lines else ""
fails = [l for l in lines if l.startswith("FAILED")][:20]
with open(out, "a") as f:
    f.write(json.dumps({"lib": lib, "parity": "pass" if rc == "0" else "fail", "tests": tests.split(),
                        "summary": summary, "failed": fails}) + "\n")
print(lib, "parity", "pass" if rc == "0" else "fail", summary)
PY
rm -f "$LOG"
[ "$RC" -eq 0 ] || [ "$RC" -eq 1 ]  # a test failure is a recorded result; a crash / timeout stops the A/B
