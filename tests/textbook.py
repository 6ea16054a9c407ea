"""Independent textbook Internet checksum (RFC 768 / RFC 793 / RFC 8200 §8.1).

Written from the RFCs, not from the reference: 16-bit words in NETWORK byte
order over the pseudo-header followed by the L4 segment, zero-padded to an
even length, folded with end-around carry, complemented.  The reference
returns the same value in native little-endian order, i.e. byte-swapped
(the Internet checksum is byte-order independent, RFC 1071 §2(B)).
Used as a second, independent check on the oracle's L4 restatement.
"""
from __future__ import annotations

import struct


def ones_sum_be(data: bytes) -> int:
    if len(data) % 2:
        data = data + b"\x00"
    s = sum(struct.unpack(f">{len(data) // 2}H", data)) if data else 0
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def rfc_checksum_be(data: bytes) -> int:
    return (~ones_sum_be(data)) & 0xFFFF


def bswap16(x: int) -> int:
    return ((x & 0xFF) << 8) | (x >> 8)


def l4_checksum_native(pkt: bytes, isv6: bool, istcp: bool, csum_start: int) -> int:
    """calc_l4_checksum semantics (generate/verify) via the RFC definition."""
    if isv6:
        src, dst = pkt[8:24], pkt[24:40]
    else:
        src, dst = pkt[12:16], pkt[16:20]
    seg = pkt[csum_start:]
    l4len = (len(pkt) - csum_start) & 0xFFFF
    if isv6:
        pseudo = src + dst + struct.pack(">I", l4len) + b"\x00\x00\x00" + bytes([6 if istcp else 17])
    else:
        pseudo = src + dst + b"\x00" + bytes([6 if istcp else 17]) + struct.pack(">H", l4len)
    return bswap16(rfc_checksum_be(pseudo + seg))


def ip_header_checksum_native(hdr: bytes) -> int:
    return bswap16(rfc_checksum_be(hdr))
