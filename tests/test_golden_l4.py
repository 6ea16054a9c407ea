"""calc_l4_checksum golden vectors from the reference's OWN checksum.cpp.

tests/golden/l4/ holds the results of /root/reference/checksum.cpp:8-36,
compiled UNCHANGED against this repository's drop-in header
(include/wireglider/checksum.hpp standing where include/netio/checksum.hpp
stood; oracle/Makefile `ref`), over 375 seeded v4/v6 x TCP/UDP packets in
generate and verify mode (tests/golden/gen_l4_golden.py; SURVEY §8(c) golden
vectors, item 2).  CPU tests: the fixtures' integrity, the oracle and the
drop-in's exported wireglider::calc_l4_checksum against them, and — where
/root/reference is mounted — that the reference's checksum.cpp still compiles
unchanged against the header, exports the symbol libwireglider_amd.so
exports, and regenerates the fixtures bit for bit.  The GPU entry points are
checked against the same fixtures in tests/test_gpu_golden_l4.py.
"""
import hashlib
import json
import os
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle

ROOT = Path(__file__).resolve().parents[1]
GOLD = ROOT / "tests" / "golden" / "l4"
REF = Path("/root/reference")
LIB = ROOT / "wireglider_amd" / "lib" / "libwireglider_amd.so"


def load():
    """(packet bytes, descriptors, kind bits, expected results, manifest)"""
    buf = np.fromfile(GOLD / "packets.bin", dtype=np.uint8)
    d = np.fromfile(GOLD / "desc.bin", dtype=oracle.PKT_DESC)
    kind = np.fromfile(GOLD / "kind.u8", dtype=np.uint8)
    exp = np.fromfile(GOLD / "expected.u16", dtype="<u2")
    return buf, d, kind, exp, json.loads((GOLD / "manifest.json").read_text())


def test_fixture_integrity():
    buf, d, kind, exp, man = load()
    for name in ("packets.bin", "desc.bin", "kind.u8", "expected.u16"):
        assert hashlib.sha256((GOLD / name).read_bytes()).hexdigest() == man[name], name
    n = man["records"]
    assert d.size == kind.size == exp.size == n
    assert np.all(d["offset"] + d["len"] <= buf.size)
    amin = np.where(d["flags"] & 1, 40, 20)
    assert np.all(d["len"] >= amin) and np.all(d["csum_start"] <= d["len"])  # the reference's contract
    assert np.any(d["csum_start"] & 1) and np.any(d["offset"] & 1)  # odd csum_start, odd placement
    assert np.any(d["len"] - d["csum_start"] > 65535)  # l4Len wrap
    # verify mode: valid packets check to 0, corrupted ones do not
    assert np.all(exp[kind == 3] == 0) and np.all(exp[kind == 7] != 0)


def test_oracle_matches_reference_checksum_cpp():
    buf, d, _, exp, _ = load()
    np.testing.assert_array_equal(oracle.l4_desc(buf, d), exp)
    for k in range(0, d.size, 7):  # the scalar entry too
        o, n = int(d["offset"][k]), int(d["len"][k])
        assert oracle.calc_l4_checksum(buf[o:o + n], bool(d["flags"][k] & 1), bool(d["flags"][k] & 2),
                                       int(d["csum_start"][k])) == exp[k]


def test_dropin_export_matches_reference_checksum_cpp(tmp_path):
    """The library's exported wireglider::calc_l4_checksum (the reference's
    mangled name, answered by the header's host path) on every record."""
    exe = tmp_path / "dropin_l4"
    subprocess.run(["g++", "-std=c++20", "-O2", f"-I{ROOT / 'include'}", str(ROOT / "tests" / "cpp" / "dropin_l4.cpp"),
                    f"-L{LIB.parent}", "-lwireglider_amd", f"-Wl,-rpath,{LIB.parent}", "-o", str(exe)], check=True)
    buf, d, _, exp, _ = load()
    blob = b"".join(struct.pack("<IBBH", int(x["len"]), int(x["flags"] & 1), int((x["flags"] >> 1) & 1),
                                int(x["csum_start"])) + buf[int(x["offset"]): int(x["offset"]) + int(x["len"])].tobytes()
                    for x in d)
    env = {k: v for k, v in os.environ.items() if k != "WG_PERCALL"}
    r = subprocess.run([str(exe)], input=blob, capture_output=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr.decode()
    got = np.array([int(x, 16) for x in r.stdout.decode().split()], dtype=np.uint16)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.skipif(not (REF / "checksum.cpp").exists(), reason="/root/reference is not mounted (GPU box)")
def test_reference_checksum_cpp_compiles_unchanged_and_regenerates(tmp_path):
    """INTEGRATION.md §2's claim as a test: the reference's own checksum.cpp
    compiles unchanged against include/wireglider/checksum.hpp, defines the
    very symbol libwireglider_amd.so exports, and reproduces the committed
    fixtures bit for bit."""
    subprocess.run(["make", "-C", str(ROOT / "oracle"), "ref"], check=True, capture_output=True)
    obj = ROOT / "oracle" / "_ref" / "ref_checksum.o"
    defined = subprocess.run(["nm", "--defined-only", str(obj)], capture_output=True, text=True, check=True).stdout
    sym = json.loads((GOLD / "manifest.json").read_text())["reference_symbol"]
    assert f" T {sym}" in defined
    exported = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True, text=True,
                              check=True).stdout
    assert f" T {sym}" in exported
    out = tmp_path / "r.u16"
    subprocess.run([str(ROOT / "oracle" / "_ref" / "ref_l4"), str(GOLD / "packets.bin"), str(GOLD / "desc.bin"),
                    str(out)], check=True)
    assert out.read_bytes() == (GOLD / "expected.u16").read_bytes()
