"""The C++ drop-in end to end on the GPU: a program compiled against
include/wireglider/checksum.hpp and linked to libwireglider_amd.so through the
reference's symbol wireglider::calc_l4_checksum (checksum.cpp:8), with
WG_PERCALL=gpu (every call through the host-memory GPU path), returns the
RFC textbook checksum for every packet, and verify-to-zero holds for the
reference test's packets (tests/test-checksum.cpp:53-82); the library's
placement counters (wg_percall_stats) show every call answered by the GPU,
none by the host fallback.  The per-call
latency of both placements is printed for DESIGN.md."""
import json
import os
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

import pktbuild
import textbook

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def build(tmp_path):
    exe = tmp_path / "dropin_l4"
    lib = ROOT / "wireglider_amd" / "lib"
    subprocess.run(["g++", "-std=c++20", "-O2", f"-I{ROOT / 'include'}", str(ROOT / "tests" / "cpp" / "dropin_l4.cpp"),
                    f"-L{lib}", "-lwireglider_amd", f"-Wl,-rpath,{lib}", "-o", str(exe)], check=True)
    return exe


def test_dropin_calc_l4_checksum_on_gpu(gpu, tmp_path):
    exe = build(tmp_path)
    rng = np.random.default_rng(2024)
    recs, exp = [], []
    stream = np.fromfile(ROOT / "tests" / "golden" / "ref" / "create_packet_65536.bin", dtype=np.uint8)
    for isv6 in (False, True):
        for istcp in (True, False):
            a = pktbuild.ipv6_addr if isv6 else pktbuild.ipv4_addr
            s, d = ("2001:db8::2", "2001:db8::1") if isv6 else ("192.0.2.2", "192.0.2.1")
            p = pktbuild.build(isv6, istcp, stream[:100].tobytes(), a(s), a(d), 1, 1)
            recs.append((p, isv6, istcp, 40 if isv6 else 20))
            exp.append(0)  # valid packet verifies to 0
    for _ in range(200):
        isv6, istcp = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
        n = int(rng.integers(40 if isv6 else 20, 3000))
        p = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        cs = int(rng.integers(0, n + 1))
        recs.append((p, isv6, istcp, cs))
        exp.append(textbook.l4_checksum_native(p, isv6, istcp, cs))
    blob = b"".join(struct.pack("<IBBH", len(p), v6, tcp, cs) + p for p, v6, tcp, cs in recs)
    r = subprocess.run([str(exe)], input=blob, capture_output=True, timeout=300,
                       env=dict(os.environ, WG_PERCALL="gpu"))
    assert r.returncode == 0, r.stderr.decode()
    got = [int(x, 16) for x in r.stdout.decode().split()]
    assert got == exp
    # every call was answered by the GPU round trip: none fell back to the
    # host (which would give the same checksums by construction)
    stats = dict(kv.split("=") for kv in r.stderr.decode().split("percall ")[-1].split())
    assert stats == {"gpu": str(len(recs)), "fallback": "0", "host": "0"}, stats
    # and the default placement answers on the host, with no GPU round trip
    r = subprocess.run([str(exe)], input=blob, capture_output=True, timeout=300,
                       env={k: v for k, v in os.environ.items() if k != "WG_PERCALL"})
    assert r.returncode == 0 and [int(x, 16) for x in r.stdout.decode().split()] == exp
    stats = dict(kv.split("=") for kv in r.stderr.decode().split("percall ")[-1].split())
    assert stats == {"gpu": "0", "fallback": "0", "host": str(len(recs))}, stats


def test_percall_latency_both_placements(gpu, tmp_path):
    exe = tmp_path / "percall_latency"
    lib = ROOT / "wireglider_amd" / "lib"
    subprocess.run(["g++", "-std=c++20", "-O2", f"-I{ROOT / 'include'}",
                    str(ROOT / "tests" / "cpp" / "percall_latency.cpp"), f"-L{lib}", "-lwireglider_amd",
                    f"-Wl,-rpath,{lib}", "-o", str(exe)], check=True)
    res = {}
    for mode, reps in (("host", 20000), ("gpu", 500)):
        env = {k: v for k, v in os.environ.items() if k != "WG_PERCALL"}
        if mode == "gpu":
            env["WG_PERCALL"] = "gpu"
        r = subprocess.run([str(exe), str(reps)], capture_output=True, text=True, timeout=300, env=env, check=True)
        res[mode] = json.loads(r.stdout)
    print("percall_latency", json.dumps(res))
    assert res["host"]["results"] == res["gpu"]["results"]  # same answers from both placements
    assert res["host"]["ns_per_call_1500B"] < res["gpu"]["ns_per_call_1500B"]
