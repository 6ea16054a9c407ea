"""Parity of the gfx950 checksum kernels against the oracle, through the C ABI.

Bit-exact (integer path): every result must equal the oracle's
calc_l4_checksum / checksum on the same bytes.  Covers the reference test
inputs (golden vectors), uniform PacketBatch geometry sweeps with arbitrary
base alignment and short last segments, random descriptor batches (odd
offsets, odd csum_start, csum_start >= len, empty packets), and the BASELINE
configs at full size with size-independent properties (generate -> store ->
verify == 0 everywhere) plus a full-array comparison against the oracle.
"""
import json
from pathlib import Path

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

GOLD = Path(__file__).resolve().parent / "golden" / "ref"


def _wga():
    import wireglider_amd

    return wireglider_amd


def to_dev(a: np.ndarray, dev, pad_front: int = 0):
    """Upload bytes to a device buffer at byte offset pad_front (arbitrary
    alignment); returns (backing tensor, view)."""
    import torch

    back = torch.zeros(a.size + pad_front + 64, dtype=torch.uint8, device=dev)
    view = back[pad_front:pad_front + a.size]
    view.copy_(torch.from_numpy(np.ascontiguousarray(a)))
    return back, view


def desc_dev(desc: np.ndarray, dev):
    import torch

    raw = np.ascontiguousarray(desc).view(np.int64).reshape(-1, 2)
    return torch.from_numpy(raw.copy()).to(dev)


def test_reference_golden_vectors(gpu):
    """tests/test-checksum.cpp:11-25 inputs through the GPU, every alignment."""
    import torch

    wga = _wga()
    stream = np.fromfile(GOLD / "create_packet_65536.bin", dtype=np.uint8)
    gold = np.fromfile(GOLD / "ref1_random_1_1500.u16", dtype="<u2")
    carry_gold = np.fromfile(GOLD / "ref1_carry_1_63.u16", dtype="<u2")
    for pad in range(16):
        back, view = to_dev(stream, gpu, pad)
        d = np.zeros(1500, dtype=oracle.PKT_DESC)
        d["offset"] = 0
        d["len"] = np.arange(1, 1501)
        out = wga.checksum_desc(view, desc_dev(d, gpu))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), gold, err_msg=f"pad {pad}")
        d1 = np.zeros(1, dtype=oracle.PKT_DESC)
        d1["len"] = 65536
        out = wga.checksum_desc(view, desc_dev(d1, gpu))
        assert int(out.cpu().numpy()[0]) == int(np.fromfile(GOLD / "ref1_random_65536.u16", dtype="<u2")[0])
    # create_packet_carry(n), n = 1..63, packed back to back at odd offsets
    bufs, offs = [], []
    o = 3
    blob = np.zeros(64 * 70 + 16, np.uint8)
    for n in range(1, 64):
        p = np.full(n, 0xFF, np.uint8)
        p[-1] = 1
        blob[o:o + n] = p
        offs.append(o)
        o += n + 1
    back, view = to_dev(blob, gpu, 5)
    d = np.zeros(63, dtype=oracle.PKT_DESC)
    d["offset"] = offs
    d["len"] = np.arange(1, 64)
    out = wga.checksum_desc(view, desc_dev(d, gpu)).cpu().numpy()
    np.testing.assert_array_equal(out, carry_gold)


SEGS = [1, 7, 20, 21, 28, 40, 48, 59, 64, 100, 127, 128, 1460, 1500, 1501, 4096, 9000, 9001]


@pytest.mark.parametrize("seg", SEGS)
def test_uniform_geometry_sweep(gpu, seg):
    import torch

    wga = _wga()
    rng = np.random.default_rng(seg)
    for trial in range(6):
        nseg = int(rng.integers(1, 40))
        total = seg * nseg - int(rng.integers(0, seg))  # short last segment
        total = max(total, 1)
        buf = rng.integers(0, 256, total, dtype=np.uint8)
        pad = int(rng.integers(0, 16))
        cs = int(rng.choice([0, 1, 20, 21, 40, 41, seg, seg + 3, int(rng.integers(0, seg + 1))]))
        flags = int(rng.integers(0, 4))
        back, view = to_dev(buf, gpu, pad)
        out = wga.calc_l4_checksum_batch(view, seg, bool(flags & 1), bool(flags & 2), cs)
        torch.cuda.synchronize()
        exp = oracle.l4_uniform(buf, seg, cs, flags)
        np.testing.assert_array_equal(out.cpu().numpy(), exp,
                                      err_msg=f"seg={seg} total={total} pad={pad} cs={cs} flags={flags}")


DESC_VARIANTS = [{"l4_small": 0}, {"l4_small": 0, "l4_nt": 0}, {"l4_small": 5}, {"l4_small": 5, "l4_nt": 0},
                 {"l4_small": 5, "lane_coop": 0}, {"l4_small": 5, "lane_coop": 0, "l4_unroll": 4},
                 {"l4_small": 5, "l4_unroll": 4},
                 {"l4_coop": 1 << 20, "l4_coop_waves": 2}, {"l4_coop": 1 << 20, "l4_coop_waves": 4, "l4_unroll": 4},
                 {"l4_coop": 1 << 20, "l4_coop_waves": 8, "l4_nt": 0}, {"l4_coop": 1 << 20, "l4_coop_waves": 16}]


@pytest.mark.parametrize("knobs", DESC_VARIANTS, ids=lambda k: ",".join(f"{a}={b}" for a, b in k.items()))
def test_desc_random(gpu, knobs):
    """Random descriptor batches under each launch variant of the kernel
    (occupancy target, descriptor mode, iterations per wave: speed knobs that
    must not change any result)."""
    import torch

    wga = _wga()
    saved = {k: wga.tune_get(k) for k in ("l4_blocks", "l4_small", "l4_nt", "l4_coop", "l4_coop_waves", "l4_unroll",
                                          "lane_coop")}
    for k, v in knobs.items():
        wga.tune_set(k, v)
    rng = np.random.default_rng(1234)
    n = 20000
    lens = rng.integers(0, 9100, n)
    lens[::97] = 0
    lens[1::89] = rng.integers(1, 40, lens[1::89].size)
    offs = np.cumsum(np.concatenate([[int(rng.integers(0, 16))], lens[:-1] + rng.integers(0, 5, n - 1)]))
    total = int(offs[-1] + lens[-1] + 16)
    buf = rng.integers(0, 256, total, dtype=np.uint8)
    d = np.zeros(n, dtype=oracle.PKT_DESC)
    d["offset"] = offs
    d["len"] = lens
    d["csum_start"] = np.minimum(rng.integers(0, 80, n), 65535)
    d["csum_start"][::7] = (lens[::7] + rng.integers(0, 3, lens[::7].size)).clip(0, 65535)
    d["flags"] = rng.integers(0, 4, n)
    back, view = to_dev(buf, gpu, 0)
    dd = desc_dev(d, gpu)
    out = wga.calc_l4_checksum_desc(view, dd)
    plain = wga.checksum_desc(view, dd)
    torch.cuda.synchronize()
    for k, v in saved.items():
        wga.tune_set(k, v)
    np.testing.assert_array_equal(out.cpu().numpy(), oracle.l4_desc(buf, d))
    np.testing.assert_array_equal(plain.cpu().numpy(), oracle.checksum_desc(buf, d))


@pytest.mark.parametrize("knob", [0, 2])
@pytest.mark.parametrize("seg", [1, 2, 3, 15, 16, 17, 20, 33, 40, 47, 60, 63, 64, 65])
def test_uniform_small_segments(gpu, seg, knob):
    """PacketBatches of small segments (<= 64 B go to the small-packet kernel
    unless l4_small_uniform = 0), every alignment, short last segment."""
    import torch

    wga = _wga()
    saved = wga.tune_get("l4_small_uniform")
    wga.tune_set("l4_small_uniform", knob)
    rng = np.random.default_rng(1000 + seg)
    try:
        for trial in range(8):
            nseg = int(rng.integers(1, 3000))
            total = max(1, seg * nseg - int(rng.integers(0, seg)))
            buf = rng.integers(0, 256, total, dtype=np.uint8)
            if trial == 0:
                buf[:] = 0  # all-zero segments
            pad = int(rng.integers(0, 16))
            cs = int(rng.choice([0, 1, 7, 12, 20, 21, 40, 41, seg, seg + 3]))
            flags = int(rng.integers(0, 4))
            back, view = to_dev(buf, gpu, pad)
            out = wga.calc_l4_checksum_batch(view, seg, bool(flags & 1), bool(flags & 2), cs)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy(), oracle.l4_uniform(buf, seg, cs, flags),
                                          err_msg=f"seg={seg} total={total} pad={pad} cs={cs} flags={flags}")
    finally:
        wga.tune_set("l4_small_uniform", saved)


@pytest.mark.parametrize("coop", [1, 0])
@pytest.mark.parametrize("small", [0, 5])
@pytest.mark.parametrize("seed", [5, 6])
def test_desc_small_packets(gpu, small, seed, coop):
    """Batches of mostly small packets (0-130 B, every alignment, csum_start
    inside, at and past the end, truncated pseudo-header addresses) with a few
    long ones mixed in: the thread-per-packet kernel's lane path (<= 64 B),
    its wave path (the rest) and the wave-per-packet kernel agree with the
    oracle."""
    import torch

    wga = _wga()
    saved = {k: wga.tune_get(k) for k in ("l4_small", "l4_coop", "lane_coop")}
    wga.tune_set("l4_small", small)
    wga.tune_set("l4_coop", 0)
    wga.tune_set("lane_coop", coop)
    rng = np.random.default_rng(seed)
    n = 30001
    lens = rng.integers(0, 131, n)
    lens[::53] = rng.integers(131, 3000, lens[::53].size)
    lens[::211] = 0
    lens[7::97] = 64
    lens[8::97] = 65
    offs = np.cumsum(np.concatenate([[int(rng.integers(0, 16))], lens[:-1] + rng.integers(0, 17, n - 1)]))
    total = int(offs[-1] + lens[-1] + 16)
    buf = rng.integers(0, 256, total, dtype=np.uint8)
    buf[offs[::31, None] + np.arange(8)] = 0  # some all-zero leading bytes
    d = np.zeros(n, dtype=oracle.PKT_DESC)
    d["offset"] = offs
    d["len"] = lens
    d["csum_start"] = rng.choice([0, 1, 19, 20, 21, 40, 41, 63, 64, 65], n)
    d["csum_start"][::9] = lens[::9]
    d["flags"] = rng.integers(0, 4, n)
    zl = np.nonzero(lens == 0)[0][:5]
    d["offset"][zl[:2]] = total - 16  # empty packets at the very end of the buffer
    back, view = to_dev(buf, gpu, 0)
    dd = desc_dev(d, gpu)
    out = wga.calc_l4_checksum_desc(view, dd)
    plain = wga.checksum_desc(view, dd)
    torch.cuda.synchronize()
    for k, v in saved.items():
        wga.tune_set(k, v)
    np.testing.assert_array_equal(out.cpu().numpy(), oracle.l4_desc(buf, d))
    np.testing.assert_array_equal(plain.cpu().numpy(), oracle.checksum_desc(buf, d))


def test_empty_and_errors(gpu):
    import torch

    wga = _wga()
    buf = torch.zeros(16, dtype=torch.uint8, device=gpu)
    out = torch.zeros(1, dtype=torch.uint16, device=gpu)
    assert wga.lib.wg_l4csum_uniform(buf.data_ptr(), 0, 1500, 20, 0, out.data_ptr(), None) == 0
    assert wga.lib.wg_l4csum_uniform(buf.data_ptr(), 16, 0, 20, 0, out.data_ptr(), None) == -1
    assert wga.lib.wg_l4csum_desc(buf.data_ptr(), buf.data_ptr() + 1, 1, out.data_ptr(), None) == -1
    torch.cuda.synchronize()


def _synth_uniform(wga, n, seg, mode, seed, dev):
    import torch

    buf = torch.empty(n * seg, dtype=torch.uint8, device=dev)
    wga.synth_fill(buf, seed)
    desc = wga.synth_desc_stride(n, seg, seg, mode, seed, 0, device=dev)
    wga.synth_headers(buf, desc, seed, 0)
    return buf, desc


def test_config2_full_size(gpu):
    """BASELINE config 2: 1,048,576 x 1500 B IPv4/UDP, generate then verify."""
    import torch

    wga = _wga()
    n, seg = 1 << 20, 1500
    buf, desc = _synth_uniform(wga, n, seg, 0, 0x5EED0002, gpu)
    out = wga.calc_l4_checksum_batch(buf, seg, False, False, 20)
    torch.cuda.synchronize()
    host = buf.cpu().numpy()
    exp = oracle.l4_uniform(host, seg, 20, 0)
    np.testing.assert_array_equal(out.cpu().numpy(), exp)
    # the descriptor form gives the same answers
    out_d = wga.calc_l4_checksum_desc(buf, desc)
    assert torch.equal(out_d, out)
    # generate -> store -> verify: all zero (offload.cpp:202-204 + evaluator.hpp:93)
    wga.store_l4csum(buf, desc, out)
    ver = wga.calc_l4_checksum_batch(buf, seg, False, False, 20)
    torch.cuda.synchronize()
    assert int(ver.to(torch.int32).abs().sum()) == 0
    # a flipped byte anywhere in one packet is caught
    buf[123456 * seg + 777] ^= 0x5A
    ver = wga.calc_l4_checksum_batch(buf, seg, False, False, 20).cpu().numpy()
    assert np.count_nonzero(ver) == 1 and ver[123456] != 0


def test_config5_mixed_slice(gpu):
    """BASELINE config 5 shard shape: v4/v6 x TCP/UDP mixed, stride 1500."""
    import torch

    wga = _wga()
    n, seg = 1 << 20, 1500
    buf, desc = _synth_uniform(wga, n, seg, 1, 0x5EED0005, gpu)
    out = wga.calc_l4_checksum_desc(buf, desc)
    torch.cuda.synchronize()
    d = desc.cpu().numpy().view(oracle.PKT_DESC).reshape(-1)
    assert 0.45 < np.mean(d["flags"] & 1) < 0.55 and 0.45 < np.mean((d["flags"] >> 1) & 1) < 0.55
    exp = oracle.l4_desc(buf.cpu().numpy(), d)
    np.testing.assert_array_equal(out.cpu().numpy(), exp)
    wga.store_l4csum(buf, desc, out)
    ver = wga.calc_l4_checksum_desc(buf, desc)
    torch.cuda.synchronize()
    assert int(ver.to(torch.int32).abs().sum()) == 0


def test_config4_bimodal_slice(gpu):
    """BASELINE config 4 shape: 64 B / 9000 B IPv4/UDP 50/50, packed."""
    import torch

    wga = _wga()
    n = 1 << 18
    rng = np.random.default_rng(0x5EED0004)
    lens = np.where(rng.random(n) < 0.5, 64, 9000).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)])
    total = int(offs[-1] + lens[-1])
    d = np.zeros(n, dtype=oracle.PKT_DESC)
    d["offset"], d["len"], d["csum_start"], d["flags"] = offs, lens, 20, 0
    buf = torch.empty(total + 16, dtype=torch.uint8, device=gpu)
    wga.synth_fill(buf, 0x5EED0004)
    dd = desc_dev(d, gpu)
    wga.synth_headers(buf, dd, 0x5EED0004, 0)
    out = wga.calc_l4_checksum_desc(buf, dd)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), oracle.l4_desc(buf.cpu().numpy(), d))


def test_host_memory_path(gpu):
    wga = _wga()
    rng = np.random.default_rng(99)
    for seg, total in [(1500, 1500 * 1000 - 3), (64, 64 * 333), (9000, 9000 * 17)]:
        buf = rng.integers(0, 256, total, dtype=np.uint8)
        got = wga.calc_l4_checksum_host(buf, seg, False, True, 20)
        np.testing.assert_array_equal(got, oracle.l4_uniform(buf, seg, 20, 2))


def test_results_deterministic_across_launches(gpu):
    import torch

    wga = _wga()
    buf, desc = _synth_uniform(wga, 1 << 16, 1500, 1, 42, gpu)
    a = wga.calc_l4_checksum_desc(buf, desc)
    b = wga.calc_l4_checksum_desc(buf, desc)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("coop", [0, 2, 4, 8, 16])
def test_long_packets(gpu, coop):
    """Packets past the issue phase's 2 KiB (the finish phase's long-packet
    loop), up to the 64 KiB maximum IP packet, at odd offsets, through the
    descriptor, verify and uniform entry points; coop > 0: the
    block-per-descriptor kernel with that many waves per packet."""
    import torch

    wga = _wga()
    saved = {k: wga.tune_get(k) for k in ("l4_coop", "l4_coop_waves")}
    wga.tune_set("l4_coop", 1 << 20 if coop else 0)
    if coop:
        wga.tune_set("l4_coop_waves", coop)
    rng = np.random.default_rng(65535)
    n = 600
    lens = rng.integers(2000, 65536, n)
    lens[:8] = [2047, 2048, 2049, 4095, 4096, 4097, 65534, 65535]
    offs = np.cumsum(np.concatenate([[int(rng.integers(0, 16))], lens[:-1] + rng.integers(0, 7, n - 1)]))
    buf = rng.integers(0, 256, int(offs[-1] + lens[-1] + 16), dtype=np.uint8)
    d = np.zeros(n, dtype=oracle.PKT_DESC)
    d["offset"], d["len"] = offs, lens
    d["csum_start"] = rng.choice([20, 21, 40, 41, 1000], n)
    d["flags"] = rng.integers(0, 4, n)
    back, view = to_dev(buf, gpu, 3)
    dd = desc_dev(d, gpu)
    out = wga.calc_l4_checksum_desc(view, dd)
    plain = wga.checksum_desc(view, dd)
    torch.cuda.synchronize()
    for k, v in saved.items():
        wga.tune_set(k, v)
    np.testing.assert_array_equal(out.cpu().numpy(), oracle.l4_desc(buf, d))
    np.testing.assert_array_equal(plain.cpu().numpy(), oracle.checksum_desc(buf, d))
    if coop:
        return
    seg = 65535
    total = seg * 5 - 777
    u = rng.integers(0, 256, total, dtype=np.uint8)
    back, view = to_dev(u, gpu, 5)
    out = wga.calc_l4_checksum_batch(view, seg, True, True, 40)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), oracle.l4_uniform(u, seg, 40, 3))


def test_read_probe_variants_run(gpu):
    """The read probes (bench.py's measured ceiling) over odd sizes: the
    contiguous and the kernel-shaped (segment runs) variants launch, finish
    and never store for real data; out-of-contract run sizes are rejected."""
    import torch

    wga = _wga()
    buf = torch.empty(1500 * 1001 + 16, dtype=torch.uint8, device=gpu)
    wga.synth_fill(buf, 3)
    acc = torch.zeros(1, dtype=torch.int64, device=gpu)
    for kib, run in ((1, 0), (2, 0), (8, 0), (1, 1500), (1, 64), (1, 2048), (1, 17)):
        wga.probe_read(buf, acc, kib, run_bytes=run)
    torch.cuda.synchronize()
    assert int(acc.item()) == 0
    with pytest.raises(Exception):
        wga.probe_read(buf, acc, 1, run_bytes=4096)


def test_host_pipeline_multichunk(gpu):
    """wg_l4csum_uniform_host's chunked two-stream pipeline:
    batches spanning many ~32 MiB chunks and more chunks than device slots,
    odd totals with a short last segment, a segment larger than a chunk,
    pageable and pinned (wg_host_alloc) inputs, two host threads at once,
    and a rebuild after wg_host_release — every result against the oracle."""
    import threading

    wga = _wga()
    rng = np.random.default_rng(4242)
    cases = [(1500, 1500 * 70001 - 777), (64, 64 * 1_200_001 + 5), (9000, 9000 * 12000 + 1),
             ((33 << 20) + 7, ((33 << 20) + 7) * 2 + 12345)]
    for seg, total in cases:
        buf = rng.integers(0, 256, total, dtype=np.uint8)
        cs, fl = int(rng.choice([20, 21, 40])), int(rng.integers(0, 4))
        got = wga.calc_l4_checksum_host(buf, seg, bool(fl & 1), bool(fl & 2), cs)
        np.testing.assert_array_equal(got, oracle.l4_uniform(buf, seg, cs, fl), err_msg=f"seg={seg} total={total}")
    # pinned input
    pb = wga.PinnedBuffer(1500 * 50000 + 3)
    pb.array[:] = rng.integers(0, 256, pb.nbytes, dtype=np.uint8)
    got = wga.calc_l4_checksum_host(pb.array, 1500, False, True, 20)
    np.testing.assert_array_equal(got, oracle.l4_uniform(pb.array, 1500, 20, 2))
    pb.close()
    # two threads, each with its own pipeline, concurrently
    bufs = [rng.integers(0, 256, 1500 * 40000 + k, dtype=np.uint8) for k in (11, 13)]
    res = [None, None]

    def work(k):
        for _ in range(3):
            res[k] = wga.calc_l4_checksum_host(bufs[k], 1500, bool(k), False, 20)
        wga.host_release()

    ts = [threading.Thread(target=work, args=(k,)) for k in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for k in (0, 1):
        np.testing.assert_array_equal(res[k], oracle.l4_uniform(bufs[k], 1500, 20, k))
    wga.host_release()
    got = wga.calc_l4_checksum_host(bufs[0], 1500, False, False, 20)  # rebuilt after release
    np.testing.assert_array_equal(got, oracle.l4_uniform(bufs[0], 1500, 20, 0))
