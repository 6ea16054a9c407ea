"""Parity of the gfx950 GSO split kernel (wg_gso_split) against the oracle's
do_tun_gso_split restatement (worker/offload.cpp:46-216): for every
super-buffer the status, the PacketBatch geometry, the whole output byte
range and the input buffer after the call (the reference modifies it in
place) must be identical.  Cases: the reference tests' packets
(tests/test-offload.cpp), random v4/v6 x TCP/UDP_L4 x ECN super-buffers with
random gso_size, payload length, TCP options, FIN/PSH, unaligned input and
output offsets, GSO_NONE in-place checksums, passthrough types and every
error status; then config 3 at full size through size-independent properties.
"""
import numpy as np
import pytest

import oracle
import pktbuild

pytestmark = pytest.mark.gpu

NEEDS_CSUM = 1


def _wga():
    import wireglider_amd

    return wireglider_amd


@pytest.fixture(params=[{"gso_ablate": 0, "gso_groups": 1}, {"gso_ablate": 32, "gso_groups": 1},
                        {"gso_groups": 3}, {"gso_groups": 12}, {"gso_groups": 5, "gso_waves": 8},
                        {"gso_groups": 3, "gso_spw": 2}, {"gso_groups": 2, "gso_spw": 0},
                        {"gso_groups": 12, "gso_waves": 1}, {"gso_groups": 7, "gso_waves": 2},
                        {"gso_groups": 3, "gso_spw": 1}, {"gso_groups": 2, "gso_spw": 3},
                        {"gso_groups": 1, "gso_spw": 4, "gso_waves": 2}],
                ids=["swizzled", "launch-order", "groups3", "groups12", "groups5x8", "groups3-pairs",
                     "groups2-serial", "groups12x1", "groups7x2", "groups3-pingpong", "groups2-triples",
                     "groups1x2-quads"])
def variant(request):
    """Every correct block -> (super-buffer, segment slot) mapping of the GSO
    kernel: one looping block per super-buffer (XCD-swizzled or in launch
    order) and several blocks per super-buffer (flat grid groups)."""
    wga = _wga()
    saved = {k: wga.tune_get(k) for k in ("gso_ablate", "gso_groups", "gso_waves", "gso_spw")}
    for k, v in request.param.items():
        wga.tune_set(k, v)
    yield request.param
    for k, v in saved.items():
        wga.tune_set(k, v)


def run_batch(gpu, cases, out_cap_fn=lambda c: None, seed=0):
    """cases: list of (pkt bytes, vnet dict, out_cap or None).  Lays the
    super-buffers out at random (unaligned) offsets, runs the GPU once, and
    compares each against the oracle."""
    import torch

    wga = _wga()
    rng = np.random.default_rng(seed)
    n = len(cases)
    desc = np.zeros(n, dtype=wga.GSO_DESC_DTYPE)
    in_off, out_off = 0, 0
    caps = []
    for k, (pkt, vnet, cap) in enumerate(cases):
        in_off += int(rng.integers(0, 17))
        out_off += int(rng.integers(0, 17))
        if cap is None:
            cap = len(pkt) + (len(pkt) // max(1, vnet.get("gso_size", 1)) + 2) * 200
        desc[k]["in_offset"], desc[k]["out_offset"] = in_off, out_off
        desc[k]["in_len"], desc[k]["out_cap"] = len(pkt), cap
        for f in ("flags", "gso_type", "hdr_len", "gso_size", "csum_start", "csum_offset"):
            desc[k]["vnet"][f] = vnet.get(f, 0)
        caps.append(cap)
        in_off += len(pkt)
        out_off += cap
    inbuf = np.zeros(in_off + 64, np.uint8)
    for k, (pkt, _, _) in enumerate(cases):
        o = int(desc[k]["in_offset"])
        inbuf[o:o + len(pkt)] = np.frombuffer(pkt, np.uint8)
    sentinel = 0xA5
    d_in = torch.from_numpy(inbuf.copy()).to(gpu)
    d_out = torch.full((out_off + 64,), sentinel, dtype=torch.uint8, device=gpu)
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(gpu)
    d_res = wga.gso_split(d_in, d_desc, d_out)
    torch.cuda.synchronize()
    g_in, g_out = d_in.cpu().numpy(), d_out.cpu().numpy()
    g_res = d_res.cpu().numpy().view(wga.GSO_RESULT_DTYPE)
    for k, (pkt, vnet, _) in enumerate(cases):
        st, o_in, o_out, vafter, res = oracle.gso_split(np.frombuffer(pkt, np.uint8), vnet, caps[k])
        r = g_res[k]
        ctx = f"case {k}: vnet={vnet} len={len(pkt)}"
        assert int(r["status"]) == st, ctx
        io = int(desc[k]["in_offset"])
        oo = int(desc[k]["out_offset"])
        if st != 0:
            continue
        assert int(r["passthrough"]) == res["passthrough"], ctx
        assert int(r["out_len"]) == res["out_len"], ctx
        assert int(r["segment_size"]) == res["segment_size"], ctx
        assert int(r["hdr_len"]) == vafter["hdr_len"], ctx
        assert int(r["isv6"]) == res["isv6"] and int(r["ecn"]) == res["ecn"], ctx
        np.testing.assert_array_equal(g_in[io:io + len(pkt)], o_in, err_msg="input after: " + ctx)
        if not res["passthrough"]:
            np.testing.assert_array_equal(g_out[oo:oo + len(o_out)], o_out, err_msg="output: " + ctx)
            # nothing written past the batch
            assert np.all(g_out[oo + len(o_out):oo + caps[k]] == sentinel), ctx
        else:
            assert np.all(g_out[oo:oo + caps[k]] == sentinel), ctx


def test_reference_offload_cases(gpu, variant):
    cases = []
    a4 = ("192.0.2.1", "192.0.2.2")
    a6 = ("2001:db8::1", "2001:db8::2")
    for hdr in (40, 0):
        p = pktbuild.make_tcp(False, a4[0], 1, a4[1], 1, 0x18, 200, 9999)
        cases.append((p, dict(flags=1, gso_type=1, hdr_len=hdr or len(p), gso_size=100, csum_start=20,
                              csum_offset=16), None))
        p = pktbuild.make_tcp(False, a4[0], 1, a4[1], 1, 0x19, 100, 9999)
        cases.append((p, dict(flags=1, gso_type=0, hdr_len=hdr or len(p), gso_size=100, csum_start=20,
                              csum_offset=16), None))
    for hdr in (60, 0):
        p = pktbuild.make_tcp(True, a6[0], 1, a6[1], 1, 0x18, 200, 9999)
        cases.append((p, dict(flags=1, gso_type=4, hdr_len=hdr or len(p), gso_size=100, csum_start=40,
                              csum_offset=16), None))
        p = pktbuild.make_tcp(True, a6[0], 1, a6[1], 1, 0x19, 100, 9999)
        cases.append((p, dict(flags=1, gso_type=0, hdr_len=hdr or len(p), gso_size=100, csum_start=40,
                              csum_offset=16), None))
    for isv6, cs, hdr in ((False, 20, 28), (True, 40, 48)):
        a = a6 if isv6 else a4
        p = pktbuild.make_udp(isv6, a[0], 1, a[1], 1, 200)
        for h in (hdr, len(p)):
            cases.append((p, dict(flags=1, gso_type=5, hdr_len=h, gso_size=100, csum_start=cs, csum_offset=6), None))
    # ECN quirk, 4 x 1460
    p = pktbuild.build(False, True, bytes(4 * 1460), pktbuild.ipv4_addr("10.0.0.1"), pktbuild.ipv4_addr("10.0.0.2"),
                       seq=100, fill_l4=False)
    cases.append((p, dict(flags=1, gso_type=0x81, gso_size=1460, csum_start=20, csum_offset=16), None))
    run_batch(gpu, cases)


def random_case(rng):
    isv6 = bool(rng.integers(0, 2))
    kind = int(rng.integers(0, 10))
    istcp = kind < 5
    plen = int(rng.choice([0, 1, 2, 15, 16, 17, int(rng.integers(0, 3000)), int(rng.integers(0, 65000))]))
    cs = 40 if isv6 else 20
    opts = b""
    if not isv6 and rng.integers(0, 4) == 0:
        opts = bytes([1]) * (4 * int(rng.integers(1, 11)))  # IPv4 options -> csum_start 24..60
        cs += len(opts)
    al = 16 if isv6 else 4
    thl = 20
    pkt = bytearray(pktbuild.build(isv6, istcp, rng.integers(0, 256, plen, dtype=np.uint8).tobytes(),
                                   rng.integers(0, 256, al, dtype=np.uint8).tobytes(),
                                   rng.integers(0, 256, al, dtype=np.uint8).tobytes(),
                                   seq=int(rng.integers(0, 2**32)), tcp_flags=int(rng.choice([0x10, 0x18, 0x19, 0x11])),
                                   ident=int(rng.integers(0, 65536)), fill_l4=bool(rng.integers(0, 2)),
                                   ip_options=opts))
    if istcp and rng.integers(0, 3) == 0 and len(pkt) >= cs + 60:
        thl = 4 * int(rng.integers(5, 16))  # TCP options: doff 5..15 (payload bytes become options)
        pkt[cs + 12] = (thl // 4) << 4
    gso = int(rng.choice([1, 7, 100, 536, 1448, 1460, int(rng.integers(1, 9000))]))
    if kind < 5:
        gt = 4 if isv6 else 1
        if rng.integers(0, 4) == 0:
            gt |= 0x80  # ECN quirk
    elif kind < 8:
        gt = 5
    elif kind == 8:
        gt = 0  # GSO_NONE (in place if NEEDS_CSUM)
    else:
        gt = int(rng.choice([3, 2, 6, 0x85]))  # passthrough types
    vnet = dict(flags=int(rng.choice([0, 1, 1, 1])), gso_type=gt, hdr_len=int(rng.integers(0, 200)), gso_size=gso,
                csum_start=cs, csum_offset=16 if (istcp and gt != 5) else 6)
    if rng.integers(0, 12) == 0:
        vnet["csum_offset"] = int(rng.integers(0, 30))  # odd / overlapping field positions
    if rng.integers(0, 15) == 0:
        vnet["gso_size"] = 0
    cap = None
    if rng.integers(0, 15) == 0:
        cap = int(rng.integers(0, len(pkt) + 100))
    return bytes(pkt), vnet, cap


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_super_buffers(gpu, variant, seed):
    rng = np.random.default_rng(seed)
    cases = [random_case(rng) for _ in range(400)]
    run_batch(gpu, cases, seed=seed)


def _far_csum_start(rng, cs, plen, istcp=True):
    """IPv4 super-buffer whose csum_start lies `cs - 20` bytes past the IP
    header (the reference takes csum_start from the vnet header as is)."""
    base = pktbuild.build(False, istcp, rng.integers(0, 256, plen, dtype=np.uint8).tobytes(),
                          pktbuild.ipv4_addr("10.1.2.3"), pktbuild.ipv4_addr("10.3.2.1"), seq=77, fill_l4=False)
    return base[:20] + rng.integers(0, 256, cs - 20, dtype=np.uint8).tobytes() + base[20:]


def test_geometry_edges(gpu, variant):
    """Segment shapes at the kernel's edges: segments shorter than a 16-B
    chunk, thousands of segments per super-buffer, headers past the 128
    prefix bytes held in registers (csum_start 508 / 600), and last segments
    of 1..17 bytes."""
    rng = np.random.default_rng(99)
    cases = []
    for gso, plen in ((1, 7000), (3, 20000), (5, 33), (15, 16 * 97 + 1), (16, 4097), (17, 300)):
        p = pktbuild.build(False, True, rng.integers(0, 256, plen, dtype=np.uint8).tobytes(),
                           pktbuild.ipv4_addr("10.0.0.1"), pktbuild.ipv4_addr("10.0.0.2"), seq=5, fill_l4=False)
        cases.append((p, dict(flags=1, gso_type=1, gso_size=gso, csum_start=20, csum_offset=16), None))
    for tail in range(1, 18):
        p = pktbuild.build(True, False, rng.integers(0, 256, 1448 * 3 + tail, dtype=np.uint8).tobytes(),
                           pktbuild.ipv6_addr("2001:db8::5"), pktbuild.ipv6_addr("2001:db8::6"), fill_l4=False)
        cases.append((p, dict(flags=1, gso_type=5, gso_size=1448, csum_start=40, csum_offset=6), None))
    for cs in (508, 600):
        p = _far_csum_start(rng, cs, 5000)
        cases.append((p, dict(flags=1, gso_type=1, gso_size=1000, csum_start=cs, csum_offset=16), None))
    # segments of 8-16 KB (near and past 8,162 / 12,258 / 16,354 B, once a
    # row-order kernel's tile limits), 16-100-B segments by the hundred, and
    # headers of 88 / 92 / 128 / 129 bytes (IPv4 options + TCP options)
    for cap in (8192, 12288, 16384):
        for seg in (cap - 30, cap - 29, (cap - 30) // 2, (cap - 30) // 2 + 1):
            p = pktbuild.build(False, True, rng.integers(0, 256, 3 * (seg - 40) + 5, dtype=np.uint8).tobytes(),
                               pktbuild.ipv4_addr("10.9.0.1"), pktbuild.ipv4_addr("10.9.0.2"), seq=9, fill_l4=False)
            cases.append((p, dict(flags=1, gso_type=1, gso_size=seg - 40, csum_start=20, csum_offset=16), None))
    for gso in (16, 17, 31, 100):
        p = pktbuild.build(False, False, rng.integers(0, 256, 40 * gso + 3, dtype=np.uint8).tobytes(),
                           pktbuild.ipv4_addr("10.9.0.3"), pktbuild.ipv4_addr("10.9.0.4"), fill_l4=False)
        cases.append((p, dict(flags=1, gso_type=5, gso_size=gso, csum_start=20, csum_offset=6), None))
    for ipopt in (8, 12):  # IPv4 options: csum_start 28 / 32, TCP doff 15 -> hdr_len 88 / 92
        opts = bytes([1]) * ipopt
        pkt = bytearray(pktbuild.build(False, True, rng.integers(0, 256, 6000, dtype=np.uint8).tobytes(),
                                       pktbuild.ipv4_addr("10.9.0.5"), pktbuild.ipv4_addr("10.9.0.6"), seq=3,
                                       fill_l4=False, ip_options=opts))
        cs = 20 + ipopt
        pkt[cs + 12] = 15 << 4
        cases.append((bytes(pkt), dict(flags=1, gso_type=1, gso_size=700, csum_start=cs, csum_offset=16), None))
    for cs in (68, 69):  # csum_start past the IP header: hdr_len 128 / 129 (the register / general header paths)
        p = _far_csum_start(rng, cs, 9000)
        pkt = bytearray(p)
        pkt[cs + 12] = 15 << 4
        cases.append((bytes(pkt), dict(flags=1, gso_type=1, gso_size=1460, csum_start=cs, csum_offset=16), None))
    run_batch(gpu, cases, seed=7)
    run_batch(gpu, cases, seed=8)


def test_config3_full_size_properties(gpu):
    """BASELINE config 3: 262,144 x (IPv4 20 + TCP 20 + 65495 B) -> 45 x 1460 B
    segments each.  Properties at full size: every segment's IPv4 header and
    L4 checksum verify (wg_checksum_desc / wg_l4csum_uniform == 0), payload
    bytes equal the input payload, and a sample of super-buffers equals the
    oracle byte for byte."""
    import torch

    wga = _wga()
    n, in_stride, out_stride = 262144, 65536, 73216
    in_len, hl, gso = 65535, 40, 1460
    nseg = (in_len - hl + gso - 1) // gso
    out_len = in_len - hl + nseg * hl
    seed = 0x5EED0003
    d_in = torch.empty(n * in_stride, dtype=torch.uint8, device=gpu)
    wga.synth_fill(d_in, seed)
    pd = np.zeros(n, dtype=wga.PKT_DESC_DTYPE)
    pd["offset"] = np.arange(n, dtype=np.uint64) * in_stride
    pd["len"], pd["csum_start"], pd["flags"] = in_len, 20, 2
    d_pd = torch.from_numpy(pd.view(np.uint8).copy()).to(gpu)
    wga.synth_headers(d_in, d_pd, seed, 0)
    desc = np.zeros(n, dtype=wga.GSO_DESC_DTYPE)
    desc["in_offset"] = pd["offset"]
    desc["out_offset"] = np.arange(n, dtype=np.uint64) * out_stride
    desc["in_len"], desc["out_cap"] = in_len, out_stride
    desc["vnet"]["flags"], desc["vnet"]["gso_type"], desc["vnet"]["gso_size"] = 1, 1, gso
    desc["vnet"]["csum_start"], desc["vnet"]["csum_offset"] = 20, 16
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(gpu)
    sample = [0, 1, 77777, n - 1]
    host_in = {b: d_in[b * in_stride:b * in_stride + in_len].cpu().numpy() for b in sample}
    d_out = torch.empty(n * out_stride, dtype=torch.uint8, device=gpu)
    res = wga.gso_split(d_in, d_desc, d_out)
    torch.cuda.synchronize()
    r = res.cpu().numpy().view(wga.GSO_RESULT_DTYPE)
    assert np.all(r["status"] == 0) and np.all(r["out_len"] == out_len) and np.all(r["segment_size"] == hl + gso)
    # verify every segment: view the outputs as one descriptor batch of segments
    sd = np.zeros(n * nseg, dtype=wga.PKT_DESC_DTYPE)
    base = (np.arange(n, dtype=np.uint64) * out_stride)[:, None] + np.arange(nseg, dtype=np.uint64)[None, :] * (hl + gso)
    sd["offset"] = base.reshape(-1)
    lens = np.full((n, nseg), hl + gso, np.uint32)
    lens[:, -1] = out_len - (nseg - 1) * (hl + gso)
    sd["len"], sd["csum_start"], sd["flags"] = lens.reshape(-1), 20, 2
    d_sd = torch.from_numpy(sd.view(np.uint8).copy()).to(gpu)
    l4 = wga.calc_l4_checksum_desc(d_out, d_sd)
    ih = sd.copy()
    ih["len"] = 20
    ipc = wga.checksum_desc(d_out, torch.from_numpy(ih.view(np.uint8).copy()).to(gpu))
    torch.cuda.synchronize()
    assert int(l4.to(torch.int32).abs().sum()) == 0
    assert int(ipc.to(torch.int32).abs().sum()) == 0
    for b in sample:
        st, o_in, o_out, _, _ = oracle.gso_split(host_in[b], dict(flags=1, gso_type=1, gso_size=gso, csum_start=20,
                                                                  csum_offset=16), out_stride)
        assert st == 0
        np.testing.assert_array_equal(d_out[b * out_stride:b * out_stride + out_len].cpu().numpy(), o_out)
        np.testing.assert_array_equal(d_in[b * in_stride:b * in_stride + in_len].cpu().numpy(), o_in)


def test_high_addresses(gpu):
    """Super-buffers spread over a 4.3 GB input, so their addresses take both
    values of bit 31 and cross the 4 GiB line: in-place (GSO_NONE +
    NEEDS_CSUM), split TCP and UDP cases each at several far offsets.  (An
    address narrowed through a signed 32-bit lane read once turned into a
    wild pointer only for buffers above such a line.)"""
    import torch

    wga = _wga()
    rng = np.random.default_rng(4242)
    span = (1 << 32) + (1 << 22)
    d_in = torch.zeros(span, dtype=torch.uint8, device=gpu)
    # bases at least 3 x 4 KiB apart (three cases of < 4 KiB each per base)
    offs = [0, 3 << 29, (1 << 31) - 6144, (1 << 31) + 16384, 3 << 30, (1 << 32) - 12288, (1 << 32) + 16384]
    cases = []
    for k, base in enumerate(offs):
        for kind in range(3):
            o = base + kind * 4096 + int(rng.integers(0, 16))
            isv6 = bool((k + kind) & 1)
            if kind == 2:
                p = pktbuild.build(isv6, False, rng.integers(0, 256, 1400, dtype=np.uint8).tobytes(),
                                   *(2 * [bytes(16 if isv6 else 4)]), fill_l4=False)
                vnet = dict(flags=1, gso_type=5, gso_size=500, csum_start=40 if isv6 else 20, csum_offset=6)
            else:
                p = pktbuild.build(isv6, True, rng.integers(0, 256, 1800, dtype=np.uint8).tobytes(),
                                   *(2 * [bytes(16 if isv6 else 4)]), seq=7, fill_l4=False)
                vnet = dict(flags=1, gso_type=(0 if kind == 0 else (4 if isv6 else 1)), gso_size=700,
                            csum_start=40 if isv6 else 20, csum_offset=16)
            cases.append((o, p, vnet))
    n = len(cases)
    desc = np.zeros(n, dtype=wga.GSO_DESC_DTYPE)
    cap = 4096
    for k, (o, p, vnet) in enumerate(cases):
        desc[k]["in_offset"], desc[k]["out_offset"] = o, k * cap
        desc[k]["in_len"], desc[k]["out_cap"] = len(p), cap
        for f in ("flags", "gso_type", "gso_size", "csum_start", "csum_offset"):
            desc[k]["vnet"][f] = vnet[f]
        d_in[o:o + len(p)] = torch.from_numpy(np.frombuffer(p, np.uint8).copy()).to(gpu)
    d_out = torch.full((n * cap,), 0xA5, dtype=torch.uint8, device=gpu)
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(gpu)
    d_res = wga.gso_split(d_in, d_desc, d_out)
    torch.cuda.synchronize()
    g_out = d_out.cpu().numpy()
    g_res = d_res.cpu().numpy().view(wga.GSO_RESULT_DTYPE)
    for k, (o, p, vnet) in enumerate(cases):
        st, o_in, o_out, vafter, res = oracle.gso_split(np.frombuffer(p, np.uint8), vnet, cap)
        r = g_res[k]
        assert int(r["status"]) == st == 0, k
        assert int(r["out_len"]) == res["out_len"], k
        np.testing.assert_array_equal(d_in[o:o + len(p)].cpu().numpy(), o_in, err_msg=f"case {k} input after")
        assert int(r["passthrough"]) == res["passthrough"], k
        if not res["passthrough"]:
            np.testing.assert_array_equal(g_out[k * cap:k * cap + res["out_len"]], o_out[:res["out_len"]],
                                          err_msg=f"case {k} output")
    del d_in
    torch.cuda.empty_cache()


def test_oversize_super_buffers(gpu):
    """in_len > 65,535 (out of contract: tun never delivers it) -> status -3
    for split and in-place candidates, input untouched; passthrough types
    still pass through.  Documented in include/wireglider_amd.h."""
    import torch

    wga = _wga()
    rng = np.random.default_rng(5)
    p4 = pktbuild.build(False, True, rng.integers(0, 256, 70000, dtype=np.uint8).tobytes(),
                        pktbuild.ipv4_addr("10.0.0.1"), pktbuild.ipv4_addr("10.0.0.2"), fill_l4=False)
    cases = [(1, 1), (0, 1), (3, 1), (0, 0)]  # (gso_type, flags): TCPv4 split, in place, passthrough x2
    n = len(cases)
    desc = np.zeros(n, dtype=wga.GSO_DESC_DTYPE)
    cap = 200000
    for k, (gt, fl) in enumerate(cases):
        desc[k]["in_offset"], desc[k]["out_offset"] = k * 80000, k * cap
        desc[k]["in_len"], desc[k]["out_cap"] = len(p4), cap
        desc[k]["vnet"]["flags"], desc[k]["vnet"]["gso_type"] = fl, gt
        desc[k]["vnet"]["gso_size"], desc[k]["vnet"]["csum_start"], desc[k]["vnet"]["csum_offset"] = 1000, 20, 16
    inbuf = np.zeros(n * 80000, np.uint8)
    for k in range(n):
        inbuf[k * 80000:k * 80000 + len(p4)] = np.frombuffer(p4, np.uint8)
    d_in = torch.from_numpy(inbuf.copy()).to(gpu)
    d_out = torch.zeros(n * cap, dtype=torch.uint8, device=gpu)
    res = wga.gso_split(d_in, torch.from_numpy(desc.view(np.uint8).copy()).to(gpu), d_out)
    torch.cuda.synchronize()
    r = res.cpu().numpy().view(wga.GSO_RESULT_DTYPE)
    assert list(r["status"]) == [-3, -3, 0, 0]
    assert list(r["passthrough"][2:]) == [1, 1] and list(r["out_len"][2:]) == [len(p4)] * 2
    np.testing.assert_array_equal(d_in.cpu().numpy(), inbuf)
