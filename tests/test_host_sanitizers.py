"""Host-side sanitizer runs of the per-call drop-in (csrc/checksum.cpp, the
exported wireglider::calc_l4_checksum that worker/offload.cpp:202 calls):
AddressSanitizer + UndefinedBehaviorSanitizer over the parity records of
test_dropin_host.py, and ThreadSanitizer over the multi-threaded harness
(one worker per tun queue, wireglider.cpp:117-151; per-thread placement
slots).  The sanitized checksum.cpp object is linked ahead of the library, so
its definition is the one the harness calls; no GPU is involved (host
placement).  GPU code is never built with sanitizers here."""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent))

import oracle  # noqa: E402
import test_dropin_host as dh  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "wireglider_amd" / "lib"


def _build(tmp_path, name, san):
    exe = tmp_path / f"{name}_{san.replace(',', '_')}"
    r = subprocess.run(["g++", "-std=c++20", "-O1", "-g", f"-fsanitize={san}", "-fno-sanitize-recover=all",
                        f"-I{ROOT / 'include'}", str(ROOT / "tests" / "cpp" / f"{name}.cpp"),
                        str(ROOT / "wireglider_amd" / "csrc" / "checksum.cpp"), f"-L{LIB}", "-lwireglider_amd",
                        f"-Wl,-rpath,{LIB}", "-lpthread", "-o", str(exe)], capture_output=True, text=True)
    if r.returncode != 0 and "sanitize" in r.stderr and "not supported" in r.stderr:
        pytest.skip(f"-fsanitize={san} unavailable: {r.stderr[-200:]}")
    assert r.returncode == 0, r.stderr
    return exe


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k != "WG_PERCALL"}
    env.update(kw)
    return env


def test_dropin_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "dropin_l4", "address,undefined")
    recs = dh._records(np.random.default_rng(78))
    got = dh._run(exe, recs, _env(ASAN_OPTIONS="detect_leaks=0:abort_on_error=1"))
    exp = [oracle.calc_l4_checksum(np.frombuffer(p, np.uint8), v6, tcp, cs) for p, v6, tcp, cs in recs]
    assert got == exp


def test_percall_threads_tsan(tmp_path):
    exe = _build(tmp_path, "percall_latency", "thread")
    reps = 300
    r = subprocess.run([str(exe), str(reps), "1", "8"], capture_output=True, text=True, timeout=300,
                       env=_env(TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-2000:]
    lat = json.loads(r.stdout)
    assert lat["percall_stats"] == {"gpu": 0, "fallback": 0, "host": 9 * 3 * (1 + reps // 10 + reps)}
    assert lat["threads_8"]["results_agree"] and lat["threads_8"]["results"] == lat["threads_1"]["results"]
