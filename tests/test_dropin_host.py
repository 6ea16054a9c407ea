"""The C++ drop-in's per-call path on the CPU (no GPU needed).

wireglider::calc_l4_checksum (checksum.cpp:8-36) is exported by
libwireglider_amd.so; per-call callers (worker/offload.cpp:202,
include/worker/evaluator.hpp:64,93) are answered on the calling CPU by the
header's host::calc_l4_checksum.  Checked against the RFC textbook (in
contract) and the oracle (every input, including the out-of-contract ones the
GPU kernels define: short packets, csum_start past the end).  With
WG_PERCALL=gpu and no device the call falls back to the same host answer
instead of aborting.
"""
import os
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle
import pktbuild
import textbook

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "wireglider_amd" / "lib"


def _build(tmp_path, name):
    exe = tmp_path / name
    subprocess.run(["g++", "-std=c++20", "-O2", f"-I{ROOT / 'include'}", str(ROOT / "tests" / "cpp" / f"{name}.cpp"),
                    f"-L{LIB}", "-lwireglider_amd", f"-Wl,-rpath,{LIB}", "-o", str(exe)], check=True)
    return exe


def _records(rng):
    """(packet, isv6, istcp, csum_start) cases and the oracle's answers."""
    recs = []
    stream = np.fromfile(ROOT / "tests" / "golden" / "ref" / "create_packet_65536.bin", dtype=np.uint8)
    for isv6 in (False, True):
        for istcp in (True, False):
            a = pktbuild.ipv6_addr if isv6 else pktbuild.ipv4_addr
            s, d = ("2001:db8::2", "2001:db8::1") if isv6 else ("192.0.2.2", "192.0.2.1")
            recs.append((pktbuild.build(isv6, istcp, stream[:100].tobytes(), a(s), a(d), 1, 1), isv6, istcp,
                         40 if isv6 else 20))
    for _ in range(300):  # in contract
        isv6, istcp = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
        n = int(rng.integers(40 if isv6 else 20, 3000))
        recs.append((rng.integers(0, 256, n, dtype=np.uint8).tobytes(), isv6, istcp, int(rng.integers(0, n + 1))))
    for n in list(range(0, 45)) + [65535, 65536, 70000]:  # short packets, csum_start past the end, l4Len wrap
        for isv6 in (False, True):
            p = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            for cs in sorted({0, n // 2, min(n, 65535), min(n + 1, 65535), 20, 40, 65535}):
                recs.append((p, isv6, bool(n & 1), cs))
    return recs


def _run(exe, recs, env):
    blob = b"".join(struct.pack("<IBBH", len(p), v6, tcp, cs) + p for p, v6, tcp, cs in recs)
    r = subprocess.run([str(exe)], input=blob, capture_output=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr.decode()
    return [int(x, 16) for x in r.stdout.decode().split()]


@pytest.mark.parametrize("percall", ["", "gpu"])
def test_dropin_per_call_host(tmp_path, percall):
    import torch

    if percall == "gpu" and torch.cuda.is_available():
        pytest.skip("covered by tests/test_gpu_dropin.py on a GPU box")
    exe = _build(tmp_path, "dropin_l4")
    recs = _records(np.random.default_rng(77))
    env = {k: v for k, v in os.environ.items() if k != "WG_PERCALL"}
    if percall:
        env["WG_PERCALL"] = percall  # no device here: must fall back, not abort
    got = _run(exe, recs, env)
    exp = [oracle.calc_l4_checksum(np.frombuffer(p, np.uint8), v6, tcp, cs) for p, v6, tcp, cs in recs]
    assert got == exp
    # the in-contract cases against the independent RFC textbook
    for (p, v6, tcp, cs), g in zip(recs, got):
        if len(p) >= (40 if v6 else 20) and cs <= len(p):
            assert g == textbook.l4_checksum_native(p, v6, tcp, cs)


def test_percall_latency_host(tmp_path):
    """The host per-call path answers in well under a microsecond (the
    number DESIGN.md §2 quotes; the GPU per-call figure comes from a box)."""
    import json

    exe = _build(tmp_path, "percall_latency")
    env = {k: v for k, v in os.environ.items() if k != "WG_PERCALL"}
    r = subprocess.run([str(exe), "20000"], capture_output=True, text=True, timeout=120, env=env, check=True)
    lat = json.loads(r.stdout)
    assert lat["ns_per_call_1500B"] < 5000


def test_percall_threads_count_and_scale(tmp_path):
    """Worker threads calling the drop-in at once (one per tun queue,
    wireglider.cpp:117-151): every call is counted exactly once in the
    per-thread placement slots, exited threads included, and the results
    agree across threads.  The per-call time at 8 threads stays near the
    1-thread figure (no shared counter line; the box measures 1 vs 16)."""
    import json

    exe = _build(tmp_path, "percall_latency")
    env = {k: v for k, v in os.environ.items() if k != "WG_PERCALL"}
    reps = 20000
    threads = [1, 8]
    r = subprocess.run([str(exe), str(reps)] + [str(t) for t in threads], capture_output=True, text=True,
                       timeout=300, env=env, check=True)
    lat = json.loads(r.stdout)
    per_thread = 3 * (1 + reps // 10 + reps)
    assert lat["percall_stats"] == {"gpu": 0, "fallback": 0, "host": sum(threads) * per_thread}
    for t in threads:
        assert lat[f"threads_{t}"]["results_agree"]
        assert lat[f"threads_{t}"]["results"] == lat["threads_1"]["results"]
    # loose on a shared CI container; the tight bound is the GPU box's figure
    assert lat["threads_8"]["ns_per_call_1500B"] < 4 * lat["threads_1"]["ns_per_call_1500B"] + 200


def test_percall_count_after_thread_exit(tmp_path):
    """Calls made from a thread_local destructor that runs after the
    library's per-thread slot owner is destroyed are counted
    once each, into the exited threads' totals, and never touch the
    destroyed owner."""
    import json

    exe = _build(tmp_path, "dropin_exit")
    env = {k: v for k, v in os.environ.items() if k != "WG_PERCALL"}
    r = subprocess.run([str(exe), "4", "100", "7"], capture_output=True, text=True, timeout=120, env=env, check=True)
    got = json.loads(r.stdout)
    assert got == {"threads": 4, "calls": 100, "exit_calls": 7, "gpu": 0, "fallback": 0, "host": 4 * 107}, got
