"""The C++ drop-in end to end on the GPU: a program compiled against
include/wireglider/checksum.hpp and linked to libwireglider_amd.so through the
reference's symbol wireglider::calc_l4_checksum (checksum.cpp:8) returns the
RFC textbook checksum for every packet, and verify-to-zero holds for the
reference test's packets (tests/test-checksum.cpp:53-82)."""
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
    r = subprocess.run([str(exe)], input=blob, capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode()
    got = [int(x, 16) for x in r.stdout.decode().split()]
    assert got == exp
