"""Packet builders for tests (stand-ins for the reference tests' libtins
make_tcp / make_udp, tests/packet_tests.hpp:12-58).  Checksums are filled with
the independent textbook implementation, never with the code under test."""
from __future__ import annotations

import struct

import numpy as np

import textbook


def ipv4_addr(s: str) -> bytes:
    return bytes(int(x) for x in s.split("."))


def ipv6_addr(s: str) -> bytes:
    import ipaddress

    return ipaddress.IPv6Address(s).packed


def build(isv6: bool, istcp: bool, payload: bytes, src: bytes, dst: bytes, sport=1, dport=1, seq=0,
          tcp_flags=0x18, ttl=64, ident=1, tos=0, fill_l4=True, ip_options: bytes = b"") -> bytes:
    l4hdr_len = 20 if istcp else 8
    l4len = l4hdr_len + len(payload)
    if istcp:
        l4 = struct.pack(">HHIIBBHHH", sport, dport, seq, 0, 0x50, tcp_flags, 32768, 0, 0)
    else:
        l4 = struct.pack(">HHHH", sport, dport, l4len & 0xFFFF, 0)
    proto = 6 if istcp else 17
    if isv6:
        ip = struct.pack(">IHBB", 0x60000000 | (tos << 20), l4len & 0xFFFF, proto, ttl) + src + dst
    else:
        ihl = 5 + len(ip_options) // 4
        total = ihl * 4 + l4len
        hdr = struct.pack(">BBHHHBBH", 0x40 | ihl, tos, total & 0xFFFF, ident, 0, ttl, proto, 0) + src + dst + ip_options
        c = textbook.ip_header_checksum_native(hdr)
        ip = hdr[:10] + struct.pack("<H", c) + hdr[12:]
    pkt = bytearray(ip + l4 + payload)
    if fill_l4:
        cs = len(ip)
        c = textbook.l4_checksum_native(bytes(pkt), isv6, istcp, cs)
        off = cs + (16 if istcp else 6)
        pkt[off:off + 2] = struct.pack("<H", c)
    return bytes(pkt)


def make_tcp(isv6: bool, src, sport, dst, dport, flags, segment_size, seq) -> bytes:
    """tests/packet_tests.hpp:12-35: zero payload of segment_size bytes."""
    a = (ipv6_addr if isv6 else ipv4_addr)
    return build(isv6, True, bytes(segment_size), a(src), a(dst), sport, dport, seq, tcp_flags=flags)


def make_udp(isv6: bool, src, sport, dst, dport, segment_size) -> bytes:
    """tests/packet_tests.hpp:37-58."""
    a = (ipv6_addr if isv6 else ipv4_addr)
    return build(isv6, False, bytes(segment_size), a(src), a(dst), sport, dport)


def random_packet(rng: np.random.Generator, isv6: bool, istcp: bool, total_len: int) -> bytes:
    """A well-formed packet of exactly total_len bytes with random payload and
    addresses, L4 checksum field zero (generate mode)."""
    hdr = (40 if isv6 else 20) + (20 if istcp else 8)
    assert total_len >= hdr
    payload = rng.integers(0, 256, total_len - hdr, dtype=np.uint8).tobytes()
    al = 16 if isv6 else 4
    src = rng.integers(0, 256, al, dtype=np.uint8).tobytes()
    dst = rng.integers(0, 256, al, dtype=np.uint8).tobytes()
    return build(isv6, istcp, payload, src, dst, int(rng.integers(1, 65535)), int(rng.integers(1, 65535)),
                 int(rng.integers(0, 2**32)), fill_l4=False)
