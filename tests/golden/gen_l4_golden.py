"""Generate the calc_l4_checksum golden vectors in tests/golden/l4/ (SURVEY §8(c)
"Golden vectors", item 2) from the reference's OWN function body.

oracle/Makefile `ref` compiles /root/reference/checksum.cpp (:1-38) UNCHANGED,
where it lies, with this repository's drop-in header standing where
include/netio/checksum.hpp stood, and links it into oracle/_ref/ref_l4 (a
driver that only calls wireglider::calc_l4_checksum over a batch).  This
script builds the input packets (seeded, numpy), runs that binary twice, and
commits data only: the packets, their wg_pkt_desc records, a per-record kind
byte and the reference's 16-bit results.  The header beneath checksum.cpp is
the repository's (its primitives are pinned separately to checksum_ref1,
tests/golden/ref/); the pseudo-header composition of checksum.cpp:8-36 is the
reference's own code.

Records (all inside the reference's contract — addresses inside the packet,
csum_start <= size, checksum.cpp:17-18,27-28,35):
  * two uniform PacketBatch runs (64 x 1500-B v4/UDP, 32 x 1024-B v6/TCP),
    well-formed, generate mode (checksum field zero), at an odd start offset;
  * v4/v6 x TCP/UDP well-formed packets of 20/40-B-header minimum size and up
    (odd sizes, 64, 65, 1500, 9000), generate mode;
  * the same packets in VERIFY mode (field = the reference's generate result,
    so the result must be 0) and verify mode with one flipped payload bit;
  * random bytes with random (half of them odd) csum_start in [0, size];
  * packets of exactly the address minimum (20 B v4 / 40 B v6), csum_start 0,
    odd, and = size (empty L4 region);
  * l4Len wrap past 65,535 (checksum.cpp:23,33 truncate to uint16_t): 65,556 B
    (l4Len 65,536 -> 0) and 65,600 B packets, even and odd csum_start.
kind bits: 1 well-formed (IP gates of evaluate_packet pass, csum_start = the IP
header size), 2 verify mode, 4 corrupted.

    python tests/golden/gen_l4_golden.py
"""
import hashlib
import json
import struct
import subprocess
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
OUT = HERE / "l4"
sys.path.insert(0, str(ROOT / "tests"))
import pktbuild  # noqa: E402

PKT_DESC = np.dtype([("offset", "<u8"), ("len", "<u4"), ("csum_start", "<u2"), ("flags", "u1"),
                     ("reserved", "u1")])
K_WELL, K_VERIFY, K_CORRUPT = 1, 2, 4


def field_off(cs: int, tcp: bool) -> int:
    return cs + (16 if tcp else 6)


def records(rng):
    """[(bytes, isv6, istcp, csum_start, kind, group)]"""
    recs = []

    def well(v6, tcp, size):
        return pktbuild.random_packet(rng, v6, tcp, size)

    for _ in range(64):
        recs.append((well(False, False, 1500), False, False, 20, K_WELL, "uniform_v4_udp_1500"))
    for _ in range(32):
        recs.append((well(True, True, 1024), True, True, 40, K_WELL, "uniform_v6_tcp_1024"))
    for v6 in (False, True):
        for tcp in (True, False):
            hmin = (40 if v6 else 20) + (20 if tcp else 8)
            sizes = [hmin, hmin + 1, 61, 64, 65, 333, 1001, 1499, 1500, 9000]
            sizes += [int(x) for x in rng.integers(hmin, 3000, 6)]
            for s in sizes:
                if s >= hmin:
                    recs.append((well(v6, tcp, s), v6, tcp, 40 if v6 else 20, K_WELL, "families"))
    for _ in range(120):
        v6, tcp = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
        amin = 40 if v6 else 20
        n = int(rng.integers(amin, 3000))
        cs = int(rng.integers(0, n + 1))
        if rng.integers(0, 2):
            cs |= 1
            cs = min(cs, n)
        recs.append((rng.integers(0, 256, n, dtype=np.uint8).tobytes(), v6, tcp, cs, 0, "random_csum_start"))
    for v6 in (False, True):
        amin = 40 if v6 else 20
        p = rng.integers(0, 256, amin, dtype=np.uint8).tobytes()
        for cs in (0, amin - 1, amin):
            for tcp in (False, True):
                recs.append((p, v6, tcp, cs, 0, "address_minimum"))
    for v6, n, cs in ((False, 65556, 20), (False, 65600, 21), (True, 65600, 40)):
        recs.append((rng.integers(0, 256, n, dtype=np.uint8).tobytes(), v6, bool(n & 1) or cs == 21, cs, 0,
                     "l4len_wrap"))
    return recs


def layout(recs, rng):
    """Packets at random gaps (any alignment); each uniform run contiguous."""
    offs, o, parts = [], 3, [bytes(3)]
    prev_group = None
    for p, _, _, _, _, g in recs:
        contiguous = g.startswith("uniform") and g == prev_group
        if not contiguous:
            gap = int(rng.integers(0, 16))
            parts.append(bytes(gap))
            o += gap
        offs.append(o)
        parts.append(p)
        o += len(p)
        prev_group = g
    parts.append(bytes(16))
    return np.frombuffer(b"".join(parts), np.uint8).copy(), offs


def descs(recs, offs):
    d = np.zeros(len(recs), dtype=PKT_DESC)
    d["offset"] = offs
    d["len"] = [len(r[0]) for r in recs]
    d["csum_start"] = [r[3] for r in recs]
    d["flags"] = [(1 if r[1] else 0) | (2 if r[2] else 0) for r in recs]
    return d


def run_ref(buf, d, tmp):
    (tmp / "p.bin").write_bytes(buf.tobytes())
    (tmp / "d.bin").write_bytes(d.tobytes())
    subprocess.run([str(ROOT / "oracle" / "_ref" / "ref_l4"), str(tmp / "p.bin"), str(tmp / "d.bin"),
                    str(tmp / "r.u16")], check=True)
    return np.fromfile(tmp / "r.u16", dtype="<u2")


def main() -> None:
    import tempfile

    subprocess.run(["make", "-C", str(ROOT / "oracle"), "ref"], check=True, capture_output=True)
    rng = np.random.default_rng(0x5EED00A5)
    recs = records(rng)
    with tempfile.TemporaryDirectory() as td:
        tmp = Path(td)
        buf, offs = layout(recs, rng)
        gen = run_ref(buf, descs(recs, offs), tmp)
        # verify mode: the well-formed non-uniform packets with the reference's
        # own result stored (native order, worker/offload.cpp:203-204), a
        # quarter of them with one payload bit flipped afterwards
        extra = []
        for k, (p, v6, tcp, cs, kind, g) in enumerate(recs):
            if kind & K_WELL and g == "families":
                q = bytearray(p)
                q[field_off(cs, tcp): field_off(cs, tcp) + 2] = struct.pack("<H", int(gen[k]))
                extra.append((bytes(q), v6, tcp, cs, K_WELL | K_VERIFY, "verify"))
                if k % 4 == 0:
                    hl = cs + (20 if tcp else 8)
                    j = int(rng.integers(hl, len(q))) if len(q) > hl else cs
                    q[j] ^= 1 << int(rng.integers(0, 8))
                    extra.append((bytes(q), v6, tcp, cs, K_WELL | K_VERIFY | K_CORRUPT, "verify_corrupted"))
        recs += extra
        buf, offs = layout(recs, rng)
        d = descs(recs, offs)
        res = run_ref(buf, d, tmp)
    kind = np.array([r[4] for r in recs], np.uint8)
    assert np.all(res[kind == (K_WELL | K_VERIFY)] == 0), "verify-mode packets must check to 0"
    OUT.mkdir(exist_ok=True)
    (OUT / "packets.bin").write_bytes(buf.tobytes())
    (OUT / "desc.bin").write_bytes(d.tobytes())
    (OUT / "kind.u8").write_bytes(kind.tobytes())
    (OUT / "expected.u16").write_bytes(res.astype("<u2").tobytes())
    groups, runs = [r[5] for r in recs], []
    for g in ("uniform_v4_udp_1500", "uniform_v6_tcp_1024"):
        idx = [i for i, x in enumerate(groups) if x == g]
        runs.append({"group": g, "first": idx[0], "count": len(idx), "offset": int(offs[idx[0]]),
                     "segment_size": len(recs[idx[0]][0]), "csum_start": recs[idx[0]][3],
                     "flags": int(d["flags"][idx[0]])})
    manifest = {f.name: hashlib.sha256(f.read_bytes()).hexdigest()
                for f in sorted(OUT.iterdir()) if f.suffix in (".bin", ".u8", ".u16")}
    manifest.update({
        "records": len(recs),
        "groups": {g: groups.count(g) for g in dict.fromkeys(groups)},
        "uniform_runs": runs,
        "kind_bits": {"1": "well-formed (evaluate_packet's IP gates pass, csum_start = IP header size)",
                      "2": "verify mode (checksum field = the reference's generate result)",
                      "4": "one payload bit flipped after the field was filled"},
        "generator": "oracle/_ref/ref_l4: /root/reference/checksum.cpp:8-36 compiled unchanged (oracle/Makefile ref) "
                     "against include/wireglider/checksum.hpp; inputs from tests/golden/gen_l4_golden.py, seed 0x5EED00A5",
        "reference_symbol": "_ZN10wireglider16calc_l4_checksumESt4spanIKhLm18446744073709551615EEbbt",
    })
    (OUT / "manifest.json").write_text(json.dumps(manifest, indent=1) + "\n")
    print(json.dumps({"records": len(recs), "bytes": int(buf.size), "groups": manifest["groups"]}, indent=1))


if __name__ == "__main__":
    main()
