"""Pin the CPU oracle against the reference's own golden vectors.

tests/golden/ref/ holds the inputs and outputs of the reference's
tests/test-checksum.cpp:11-51 produced by compiling its test oracle
(tests/checksum_tests.hpp) in place (tests/golden/gen_golden.py).  The
oracle's checksum_ref1 restatement and its nofold/fold path (the
checksum.hpp contract) must reproduce every one of them.
"""
import json
from pathlib import Path

import numpy as np
import pytest

import oracle

GOLD = Path(__file__).resolve().parent / "golden" / "ref"


@pytest.fixture(scope="module")
def golden():
    return dict(
        stream=np.fromfile(GOLD / "create_packet_65536.bin", dtype=np.uint8),
        random=np.fromfile(GOLD / "ref1_random_1_1500.u16", dtype="<u2"),
        carry=np.fromfile(GOLD / "ref1_carry_1_63.u16", dtype="<u2"),
        r65536=int(np.fromfile(GOLD / "ref1_random_65536.u16", dtype="<u2")[0]),
        manifest=json.loads((GOLD / "manifest.json").read_text()),
    )


def carry_packet(n):
    """create_packet_carry (tests/checksum_tests.hpp:44-48)."""
    a = np.full(n, 0xFF, dtype=np.uint8)
    a[-1] = 1
    return a


def test_manifest_hashes(golden):
    import hashlib

    for name, h in golden["manifest"].items():
        if name.endswith((".bin", ".u16")):
            assert hashlib.sha256((GOLD / name).read_bytes()).hexdigest() == h, name


def test_anchor_values(golden):
    # SURVEY §8c anchors computed with the reference's checksum_ref1.
    r = golden["random"]
    assert [int(r[n - 1]) for n in (1, 2, 3, 20, 64, 100, 1460, 1500)] == [
        0xFF59, 0x0F59, 0x0E81, 0xF361, 0x3F6D, 0x6826, 0x01ED, 0x6406]
    assert golden["r65536"] == 0xCB6C
    assert golden["stream"][:8].tobytes().hex() == "a6f0d82981c7d7fd"


def test_ref1_restatement_random(golden):
    # tests/test-checksum.cpp:11-17 (sizes 1..1500); create_packet(n) is a prefix
    # of one deterministic stream (tests/checksum_tests.hpp:36-42).
    s = golden["stream"]
    for n in range(1, 1501):
        assert oracle.checksum_ref1(s[:n]) == golden["random"][n - 1], n


def test_checksum_equals_ref1_random(golden):
    # wireglider::checksum(create_packet(n), 0) == checksum_ref1 (test-checksum.cpp:11-17)
    s = golden["stream"]
    for n in range(1, 1501):
        assert oracle.checksum(s[:n], 0) == golden["random"][n - 1], n
    assert oracle.checksum(s, 0) == golden["r65536"]


def test_checksum_carry(golden):
    # tests/test-checksum.cpp:19-25
    for n in range(1, 64):
        p = carry_packet(n)
        assert oracle.checksum_ref1(p) == golden["carry"][n - 1]
        assert oracle.checksum(p, 0) == golden["carry"][n - 1]


@pytest.mark.parametrize("off,n", [(0, 1), (0, 2), (0, 4), (0, 8), (0, 16)])
def test_checksum_sizes(golden, off, n):
    # tests/test-checksum.cpp:35-42 (fixed extents at offset 0 of create_packet(16))
    p = golden["stream"][:16][off:off + n]
    assert oracle.fold_complement(oracle.nofold(p, 0)) == oracle.checksum_ref1(p)


@pytest.mark.parametrize("off,n", [(15, 1), (14, 2), (12, 4), (8, 8), (0, 16)])
def test_checksum_sizes_carry(off, n):
    # tests/test-checksum.cpp:44-51
    p = carry_packet(16)[off:off + n]
    assert oracle.fold_complement(oracle.nofold(p, 0)) == oracle.checksum_ref1(p)


def test_zero_vs_ffff_split():
    # all-zero data -> 0xFFFF; non-zero data summing to 0 mod 0xFFFF -> 0x0000
    assert oracle.checksum(np.zeros(100, np.uint8), 0) == 0xFFFF
    assert oracle.checksum(np.array([0xFF, 0xFF], np.uint8), 0) == 0x0000
    assert oracle.checksum(np.zeros(0, np.uint8), 0) == 0xFFFF


def test_rfc1071_example():
    # RFC 1071 §3: bytes 00 01 f2 03 f4 f5 f6 f7 -> one's-complement sum ddf2
    # (network order), checksum 220d; native little-endian result = 0x0d22.
    b = np.array([0x00, 0x01, 0xF2, 0x03, 0xF4, 0xF5, 0xF6, 0xF7], np.uint8)
    assert oracle.checksum(b, 0) == 0x0D22


def test_ipv4_header_known_answer():
    # A well-known IPv4 header (checksum field b861 in network order) must
    # verify to 0 and regenerate b861 with the field zeroed.
    hdr = bytes.fromhex("450000730000400040 11b861c0a80001c0a800c7".replace(" ", ""))
    a = np.frombuffer(hdr, np.uint8)
    assert oracle.checksum(a, 0) == 0
    z = a.copy()
    z[10:12] = 0
    c = oracle.checksum(z, 0)
    assert bytes([c & 0xFF, c >> 8]) == bytes.fromhex("b861")


def test_nofold_initial_zero_semantics():
    # nofold(b, initial) folds like the integer sum initial + words (mod 0xFFFF).
    rng = np.random.default_rng(1)
    for _ in range(200):
        n = int(rng.integers(0, 300))
        b = rng.integers(0, 256, n, dtype=np.uint8)
        init = int(rng.integers(0, 2**64, dtype=np.uint64))
        words = sum(int(b[i]) | (int(b[i + 1]) << 8) for i in range(0, n - 1, 2)) + (int(b[-1]) if n % 2 else 0)
        s = init + words
        exp = 0xFFFF if s == 0 else (~(1 + (s - 1) % 0xFFFF)) & 0xFFFF
        assert oracle.checksum(b, init) == exp


def test_vector_nofold_arm_pinned(golden):
    """The AVX2 arm of orc_nofold (the CPU baseline's fastcsum-class path,
    include/netio/checksum.hpp:88-91) against the reference goldens and the
    scalar arm: every length 256..1500 of create_packet, the 65536-B golden,
    all-0xFF carry buffers, zero buffers, odd offsets and non-zero initials."""
    assert oracle.have_avx2(), "the oracle's vector arm needs AVX2 (x86-64-v3) on this host"
    s = golden["stream"]
    for n in range(256, 1501):
        assert oracle.checksum(s[:n], 0) == golden["random"][n - 1], n
    assert oracle.checksum(s, 0) == golden["r65536"]
    rng = np.random.default_rng(11)
    for _ in range(400):
        n = int(rng.integers(256, 70000))
        o = int(rng.integers(0, 64))
        init = int(rng.integers(0, 2**64, dtype=np.uint64)) if rng.random() < 0.5 else 0
        buf = s[o:o + n] if o + n <= s.size else rng.integers(0, 256, n, dtype=np.uint8)
        if rng.random() < 0.2:
            buf = np.full(n, 0xFF, np.uint8)
        assert oracle.fold_complement(oracle.nofold(buf, init)) == oracle.fold_complement(
            oracle.nofold_scalar(buf, init))
    assert oracle.checksum(np.zeros(4096, np.uint8), 0) == 0xFFFF
    for n in (256, 257, 4095, 65536):
        assert oracle.checksum(carry_packet(n), 0) == oracle.checksum_ref1(carry_packet(n))
