#!/usr/bin/env python3
"""Benchmark: device-resident GiB/s of the L4 checksum over a packet batch.

BASELINE.json metric "device-resident GiB/s, L4 checksum over packet batch;
1/2/4/8 MI355X".  One step = one launch of the gfx950 kernel over one whole
batch already resident in HBM (reference: calc_l4_checksum, checksum.cpp:8-36,
once per segment of a PacketBatch, include/worker/offload.hpp:19-29).

Workloads (--workload; BASELINE.json configs):
  config1            checksum(buf, 0) over 16,384 x 64 KiB random buffers
                     (configs[0], tests/test-checksum.cpp:11-17 shape): the
                     CPU baseline on 1 core and all cores beside
                     wg_checksum_desc on the same bytes.
  config2 (default)  1,048,576 x 1500 B IPv4/UDP per GPU, uniform PacketBatch
                     (configs[1]); N GPUs = N independent shards, weak
                     scaling, no data-path collective.
  config3            262,144 x 64 KiB GSO super-buffers -> 45 x 1460 B TCP
                     segments per GPU (configs[2]), fused split + checksums.
  config3udp         the same super-buffers as UDP_L4 (gso_type 5, 8-B UDP
                     header) -> 45 x 1472 B UDP segments.
  config4            4,194,304 bimodal 64 B / 9000 B IPv4/UDP (configs[3]).
  config5            16,777,216 x 1500 B mixed v4/v6 x TCP/UDP split across
                     the N GPUs (configs[4]); strong scaling.
  verify             SURVEY §8 f1: decap verify gates (wg_verify_desc) over
                     1,048,576 x 1500 B mixed v4/v6 x TCP/UDP per GPU with
                     checksums stored; metric GiB/s of packets verified.
  gro                SURVEY §8 f2: GRO finalize (wg_gro_finalize) of
                     4,194,304 coalesced flows per GPU, headers in 64 B slots,
                     mixed v4/v6 x TCP/UDP; metric Mflows/s.
  aead               SURVEY §8 f4: WireGuard data-message encryption
                     (wg_aead_encrypt_batch, ChaCha20-Poly1305) of 1,048,576 x
                     1500 B packets per GPU (the encap worker's PacketBatch),
                     decrypt of the result in post_checks; metric GiB/s of
                     plaintext.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload config2]
  torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N
ranks itself (torch.distributed.run, one process per GPU) before touching the
GPU and exits with their status; every rank checks that the process group
holds exactly N ranks.
Rank 0 prints ONE JSON line.  Outside the timed region: a GPU verify pass
(store the checksums, re-run in verify mode, every result must be 0),
an RCCL all-gather of the results (timed separately) and an order-independent
result hash; rank 0 at N=1 also times the CPU oracle on a sample.  Unless
--no-strong, the line also carries `strong_scaling`: BASELINE config 5
(16,777,216 x 1500 B mixed, split across the N ranks) timed the same way, so
the driver's 1/2/4/8 runs give a weak (config 2) and a strong (config 5) curve.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import Callable, Optional

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X spec HBM3E peak (MI355X_MICROARCH.md, chip table)
SEG = 1500


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="config2",
                    choices=["config1", "config2", "config3", "config3udp", "config4", "config4small", "config4strong",
                             "config5", "verify64", "verify1500u",
                             "verify", "verify64d", "gro", "encap", "encap_2call", "aead", "encap_host", "decap_host"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-post", action="store_true",
                    help="skip the workload's own post-checks (PMC passes: only the step's launches of its kernels)")
    ap.add_argument("--no-strong", action="store_true", help="skip the config 5 strong-scaling companion")
    ap.add_argument("--force-dist", action="store_true",
                    help="create the process group (WG_DIST_BACKEND, default nccl = RCCL) even at world size 1, "
                         "so every collective of the multi-GPU path runs (the RCCL path checked on one GPU)")
    ap.add_argument("--cpu-seconds", type=float, default=2.0,
                    help="wall seconds of each CPU baseline repetition on all cores (half on one core); 8 repetitions each, the first dropped")
    ap.add_argument("--settle-seconds", type=float, default=0.3,
                    help="untimed back-to-back launches before the warmup (clock/memory settle)")
    return ap.parse_args()


@dataclass
class Workload:
    launch: Callable[[], None]
    n_units: int                 # packets (or super-buffers) on this rank
    payload_bytes: int           # bytes counted by the metric (this rank)
    alg_bytes: int               # algorithmic HBM bytes per launch (roofline numerator)
    cfg: dict
    scaling: str
    buf: object                  # the batch buffer (read-roofline probe target)
    kernel: str
    first_index: int = 0         # global index of this rank's first packet
    out: Optional[object] = None      # uint16 results (L4 workloads)
    desc: Optional[object] = None     # descriptor tensor (verify pass)
    sample: Optional[Callable] = None  # host sample for the CPU baseline
    counts: list = field(default_factory=list)  # packets per rank
    metric: Optional[str] = None      # overrides the default metric (f-row workloads)
    unit: str = "GiB/s"
    value_scale: float = 2.0**-30     # metric value = payload units/s x value_scale
    post: Optional[Callable] = None   # workload-specific post-check
    probe_run: int = 0                # packet size for the kernel-shaped read probe (0: contiguous only)
    pcie: Optional[dict] = None       # host-memory workloads: PCIe bytes per step {"h2d": B, "d2h": B}
    rw: Optional[tuple] = None        # (read, written) algorithmic bytes per launch, when both directions count
    copy_dst: Optional[object] = None  # read+write workloads: a device buffer the copy probe may overwrite
    valu_kernel: Optional[str] = None  # VALU-bound workloads: the timed kernel's full symbol (valu_issue check)


def aead_kernel_symbol(wga, maxpay: int, dec: bool = False, ver: bool = False, gso: int = 0) -> str:
    """The demangled symbol of the AEAD kernel launch_aead (csrc/aead.hip)
    picks for a batch whose largest payload is `maxpay` bytes: K blocks per
    lane (knob aead_k; 0 = 2 or 3, whichever packs a wave better), a group of
    exactly the lanes needed (template 0) up to 32, 1 lane (1), else 64."""
    nblk = (((maxpay + 15) & ~15) + 63) // 64
    K = wga.tune_get("aead_k")
    if K == 0:
        c = nblk + 1
        l2, l3 = (c + 1) // 2, (c + 2) // 3
        w2 = 64 // l2 if l2 <= 32 else 0
        w3 = 64 // l3 if l3 <= 32 else 0
        K = 3 if 2 * w3 > 3 * w2 else 2
    lanes = (nblk + 1 + K - 1) // K
    G = 1 if lanes <= 1 else (0 if lanes <= 32 else 64)
    # encrypt with exact-size groups: messages staged in LDS when a block's
    # slots fit kStageMaxBlockLds (aead.hip launch_gk)
    lds_block = 4 * (64 // lanes) * (32 + ((maxpay + 15) & ~15)) if G == 0 else 0
    stage = not dec and G == 0 and wga.tune_get("aead_stage") == 1 and lds_block <= 53248
    # wg_encap_batch with the staged kernel: header synthesis (knob encap_synth)
    syn = gso == 2 and stage and wga.tune_get("encap_synth") == 1
    b = lambda v: "true" if v else "false"
    return f"void wg::aead_kernel<{G}, {K}, {b(dec)}, {b(ver)}, {gso}, {b(stage)}, {b(syn)}>(wg::AeadParams)"


def build_workload(wga, torch, name: str, rank: int, world: int, dev) -> Workload:
    import numpy as np

    if name == "config2":
        n = 1 << 20
        seed = 0x5EED0002
        buf = torch.empty(n * SEG, dtype=torch.uint8, device=dev)
        # shard-invariant data: byte counter and packet index offset by rank
        wga.synth_fill(buf, seed, counter_base=rank * n * SEG)
        desc = wga.synth_desc_stride(n, SEG, SEG, 0, seed, rank * n, device=dev)
        wga.synth_headers(buf, desc, seed, rank * n)
        out = torch.empty(n, dtype=torch.uint16, device=dev)

        def launch():
            wga.calc_l4_checksum_batch(buf, SEG, False, False, 20, out=out)

        def sample(npk):
            return buf[: npk * SEG].cpu().numpy(), out[:npk].cpu().numpy(), ("uniform", SEG, 20, 0)

        cfg = {"workload": "config2: 1,048,576 x 1500 B IPv4/UDP per GPU, uniform PacketBatch (stride 1500)",
               "packets_per_gpu": n, "segment_size": SEG, "csum_start": 20, "layout": "uniform",
               "parallelism": f"shard{world} (independent packet shards, no data-path collective)"}
        return Workload(launch, n, n * SEG, n * SEG + 2 * n, cfg, "weak", buf, "wg::l4csum_kernel<0,4,nt>",
                        rank * n, out, desc, sample, [n] * world, probe_run=SEG)
    if name == "config5":
        from wireglider_amd import dist as wdist

        total = 1 << 24
        lo, hi = wdist.shard_bounds(total, world, rank)
        n = hi - lo
        seed = 0x5EED0005
        buf = torch.empty(n * SEG, dtype=torch.uint8, device=dev)
        wga.synth_fill(buf, seed, counter_base=lo * SEG)
        desc = wga.synth_desc_stride(n, SEG, SEG, 1, seed, lo, device=dev)
        wga.synth_headers(buf, desc, seed, lo)
        out = torch.empty(n, dtype=torch.uint16, device=dev)

        def launch():
            wga.calc_l4_checksum_desc(buf, desc, out=out)

        def sample(npk):
            return buf[: npk * SEG].cpu().numpy(), out[:npk].cpu().numpy(), ("desc", desc[:npk].cpu().numpy())

        cfg = {"workload": "config5: 16,777,216 x 1500 B mixed IPv4/IPv6 x TCP/UDP split across GPUs "
                           "(descriptor batch)",
               "packets_total": total, "packets_per_gpu": n, "segment_size": SEG, "layout": "descriptor",
               "parallelism": f"shard{world} (contiguous packet ranges, no data-path collective)"}
        counts = [wdist.shard_bounds(total, world, r)[1] - wdist.shard_bounds(total, world, r)[0]
                  for r in range(world)]
        return Workload(launch, n, n * SEG, n * SEG + 2 * n + 16 * n, cfg, "strong", buf,
                        "wg::l4csum_split_kernel<1,nt> (l4_small=5)", lo, out, desc, sample, counts, probe_run=SEG)
    if name in ("encap", "encap_2call"):
        return build_encap(wga, torch, rank, world, dev, fused=name == "encap")
    if name in ("config3", "config3udp"):
        udp = name == "config3udp"
        n, in_stride, out_stride = 1 << 18, 65536, 73216  # outbuf stride of worker/encap.cpp:26
        in_len = 65535
        # TCPV4 (doff 5, ACK|PSH): 40-B headers, gso_size 1460; UDP_L4 (gso_type 5,
        # worker/offload.cpp:113-115,197-199): 28-B headers, gso_size 1472
        hdr, gso, pflags = (28, 1472, 0) if udp else (40, 1460, 2)
        seed = 0x5EED0003
        buf = torch.empty(n * in_stride, dtype=torch.uint8, device=dev)
        wga.synth_fill(buf, seed, counter_base=rank * n * in_stride)
        pd = np.zeros(n, dtype=wga.PKT_DESC_DTYPE)
        pd["offset"] = np.arange(n, dtype=np.uint64) * in_stride
        pd["len"], pd["csum_start"], pd["flags"] = in_len, 20, pflags
        wga.synth_headers(buf, torch.from_numpy(pd.view(np.uint8).copy()).to(dev), seed, rank * n)
        gd = np.zeros(n, dtype=wga.GSO_DESC_DTYPE)
        gd["in_offset"] = pd["offset"]
        gd["out_offset"] = np.arange(n, dtype=np.uint64) * out_stride
        gd["in_len"], gd["out_cap"] = in_len, out_stride
        gd["vnet"]["flags"], gd["vnet"]["gso_type"], gd["vnet"]["gso_size"] = 1, (5 if udp else 1), gso
        gd["vnet"]["csum_start"], gd["vnet"]["csum_offset"] = 20, (6 if udp else 16)
        d_desc = torch.from_numpy(gd.view(np.uint8).copy()).to(dev)
        outb = torch.empty(n * out_stride, dtype=torch.uint8, device=dev)
        res = torch.empty(n * wga.GSO_RESULT_BYTES, dtype=torch.uint8, device=dev)
        nseg = (in_len - hdr + gso - 1) // gso
        out_len = in_len - hdr + nseg * hdr

        def launch():
            wga.gso_split(buf, d_desc, outb, results=res)

        def post():
            # size-independent properties over the whole output: every status
            # 0 with the expected geometry, and every segment's IPv4 header and
            # L4 checksum verify to 0 (wg_checksum_desc / wg_l4csum_desc)
            r = res.cpu().numpy().view(wga.GSO_RESULT_DTYPE)
            geom_bad = int(np.count_nonzero((r["status"] != 0) | (r["out_len"] != out_len)
                                            | (r["segment_size"] != hdr + gso)))
            sd = np.zeros(n * nseg, dtype=wga.PKT_DESC_DTYPE)
            base = (gd["out_offset"][:, None] + np.arange(nseg, dtype=np.uint64)[None, :] * np.uint64(hdr + gso))
            sd["offset"] = base.reshape(-1)
            lens = np.full((n, nseg), hdr + gso, np.uint32)
            lens[:, -1] = out_len - (nseg - 1) * (hdr + gso)
            sd["len"], sd["csum_start"], sd["flags"] = lens.reshape(-1), 20, pflags
            d_sd = torch.from_numpy(sd.view(np.uint8)).to(dev)
            l4 = wga.calc_l4_checksum_desc(outb, d_sd)
            sd["len"] = 20
            ipc = wga.checksum_desc(outb, torch.from_numpy(sd.view(np.uint8)).to(dev))
            torch.cuda.synchronize()
            return {"result_geometry_mismatches": geom_bad, "segments_checked": int(n * nseg),
                    "l4_verify_nonzero": int(torch.count_nonzero(l4.to(torch.int32)).item()),
                    "ipv4_header_verify_nonzero": int(torch.count_nonzero(ipc.to(torch.int32)).item())}

        def sample(_npk):
            # 4,096 super-buffers (268 MB in, 300 MB out: past the host L3),
            # their GPU output and their descriptors rebased to the sample
            k = min(n, 4096)
            gk = gd[:k].copy()
            # the sampled slots refilled with a sentinel and the batch split
            # once more (untimed): each super-buffer's PacketBatch [0, out_len)
            # is compared with the oracle, and the rest of its 73,216-B slot
            # must still hold the sentinel — a stray write there fails parity
            # (zeroing the tail before comparing hid such writes)
            outb[: k * out_stride].fill_(0xA5)
            launch()
            torch.cuda.synchronize()
            g = outb[: k * out_stride].cpu().numpy().reshape(k, out_stride)
            if np.all(g[:, out_len:] == 0xA5):
                g[:, out_len:] = 0  # the oracle's buffer is zero past out_len
            return (buf[: k * in_stride].cpu().numpy(), g.reshape(-1), ("gso", gk, k * out_stride))

        proto = ("UDP_L4, IPv4/UDP, 65535 B) -> 45 x 1472 B UDP segments each"
                 if udp else "IPv4/TCP, 65535 B) -> 45 x 1460 B segments each")
        cfg = {"workload": f"{name}: 262,144 x 64 KiB GSO super-buffers ({proto}, fused copy + header "
                           "fix-up + IPv4/L4 checksums",
               "super_buffers_per_gpu": n, "gso_size": gso, "gso_type": "UDP_L4" if udp else "TCPV4",
               "segments_per_buffer": nseg, "parallelism": f"shard{world}"}
        alg = n * in_len + n * out_len + n * (wga.GSO_DESC_BYTES + wga.GSO_RESULT_BYTES)
        return Workload(launch, n, n * in_len, alg, cfg, "weak", buf,
                        "wg::gso_plan_kernel + wg::gso_split_kernel<4,4,0> + wg::gso_finalize_kernel (one wg_gso_split call)",
                        rank * n, sample=sample, counts=[n] * world, post=post,
                        rw=(n * in_len + n * (wga.GSO_DESC_BYTES + wga.GSO_RESULT_BYTES), n * out_len),
                        copy_dst=outb)
    if name == "aead":
        # worker/encap.cpp:136-141: Peer::encrypt for every 1500-B segment of a
        # PacketBatch (config 2's packets), counters encrypt_nonce++ per call
        n = 1 << 20
        seed = 0x5EED00F4
        buf = torch.empty(n * SEG, dtype=torch.uint8, device=dev)
        wga.synth_fill(buf, seed, counter_base=rank * n * SEG)
        wga.synth_headers(buf, wga.synth_desc_stride(n, SEG, SEG, 0, seed, rank * n, device=dev), seed, rank * n)
        key = np.random.default_rng(seed).integers(0, 256, 32, dtype=np.uint8).tobytes()
        rx, c0 = 0x1A2B3C4D, (rank * n) + 1000
        mseg = wga.aead_message_stride(SEG)
        out = torch.empty(n * mseg, dtype=torch.uint8, device=dev)
        st = torch.empty(n, dtype=torch.int8, device=dev)

        def launch():
            wga.aead_encrypt_batch(buf, SEG, key, rx, c0, out=out, status=st)

        def post():
            # decrypt the messages back (worker/decap_ref.cpp:78-86), timed like
            # the main line; every status 0 and every plaintext equal to its packet
            pt = torch.empty(n * (mseg - 32), dtype=torch.uint8, device=dev)
            dst = torch.empty(n, dtype=torch.int8, device=dev)
            for _ in range(5):
                wga.aead_decrypt_batch(out, mseg, key, out=pt, status=dst)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(20):
                wga.aead_decrypt_batch(out, mseg, key, out=pt, status=dst)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            same = bool(torch.equal(pt.view(n, mseg - 32)[:, :SEG], buf.view(n, SEG)))
            res = {"encrypt_status_nonzero": int(torch.count_nonzero(st).item()),
                   "decrypt": {"kernel_ms": round(ms, 5), "GiB_s": round(n * SEG / (ms * 1e-3) / 2**30, 1),
                               "status_nonzero": int(torch.count_nonzero(dst).item()),
                               "plaintext_round_trip_equal": same}}
            del pt, dst
            res["decap_fused"] = decap_fused()
            return res

        def timed(fn, reps=20):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / reps

        def decap_fused():
            """The decap worker's decrypt + evaluate_packet (worker/decap_ref.cpp:
            81-86) on 1 M valid 1,504-B packets (a multiple of 16, so the padded
            plaintext is the IP packet and every gate runs): decrypt then
            wg_verify_desc over the plaintexts, against the fused
            wg_aead_decrypt_verify_batch (one pass, the plaintext never re-read);
            verdicts and L4 results identical."""
            s2 = 1504
            m2 = wga.aead_message_stride(s2)
            pk = torch.empty(n * s2, dtype=torch.uint8, device=dev)
            wga.synth_fill(pk, seed + 1, counter_base=rank * n * s2)
            d2 = wga.synth_desc_stride(n, s2, s2, 1, seed + 1, rank * n, device=dev)
            wga.synth_headers(pk, d2, seed + 1, rank * n)
            wga.store_l4csum(pk, d2, wga.calc_l4_checksum_desc(pk, d2))
            msgs = torch.empty(n * m2, dtype=torch.uint8, device=dev)
            wga.aead_encrypt_batch(pk, s2, key, rx, c0, out=msgs)
            del pk
            pt = torch.empty(n * (m2 - 32), dtype=torch.uint8, device=dev)
            dst = torch.empty(n, dtype=torch.int8, device=dev)
            vd = torch.empty(n, dtype=torch.uint8, device=dev)
            l4a = torch.empty(n, dtype=torch.uint16, device=dev)
            vf = torch.empty(n, dtype=torch.uint8, device=dev)
            l4f = torch.empty(n, dtype=torch.uint16, device=dev)
            t_dec = timed(lambda: wga.aead_decrypt_batch(msgs, m2, key, out=pt, status=dst))
            t_ver = timed(lambda: wga.verify_desc(pt, d2, verdict=vd, l4=l4a))  # plaintext i at i * 1504: d2
            t_fused = timed(lambda: wga.aead_decrypt_verify_batch(msgs, m2, key, out=pt, status=dst, verdict=vf,
                                                                  l4=l4f))
            equal = bool(torch.equal(vd, vf) and torch.equal(l4a, l4f))
            passing = int(torch.count_nonzero((vf & 3) == 3).item())
            return {"packets": n, "packet_bytes": s2, "decrypt_ms": round(t_dec, 5), "verify_ms": round(t_ver, 5),
                    "decrypt_plus_verify_ms": round(t_dec + t_ver, 5), "fused_ms": round(t_fused, 5),
                    "fused_GiB_s": round(n * s2 / (t_fused * 1e-3) / 2**30, 1),
                    "verdicts_equal_to_separate": equal, "packets_passing_both_gates": passing}

        def sample(npk):
            k = min(n, 1 << 16)  # ~98 MB: the scalar C oracle runs ~0.15 GB/s per core
            return buf[: k * SEG].cpu().numpy(), out[: k * mseg].cpu().numpy(), ("aead", key, rx, c0, SEG)

        cfg = {"workload": "aead (SURVEY §8 f4): WireGuard data-message encryption (ChaCha20-Poly1305, "
                           "Peer::encrypt per segment) of 1,048,576 x 1500 B packets per GPU",
               "packets_per_gpu": n, "segment_size": SEG, "message_stride": mseg, "parallelism": f"shard{world}"}
        ksym = aead_kernel_symbol(wga, SEG)
        return Workload(launch, n, n * SEG, n * SEG + n * mseg + n, cfg, "weak", buf,
                        f"{ksym} (VALU-bound: ChaCha20 + Poly1305)", rank * n, sample=sample,
                        counts=[n] * world, post=post, valu_kernel=ksym,
                        metric="device-resident GiB/s of plaintext, WireGuard data-message encryption (SURVEY f4)")
    if name == "config1":
        # tests/test-checksum.cpp:11-17: checksum(create_packet(n), 0) on random
        # buffers; BASELINE configs[0] at 64 KiB, 16,384 buffers (1 GiB,
        # past the host LLC), SURVEY §8(d).  On the GPU the same bytes go
        # through wg_checksum_desc (checksum(span, 0) per descriptor).
        n, size = 16384, 65536
        seed = 0x5EED0001
        buf = torch.empty(n * size, dtype=torch.uint8, device=dev)
        wga.synth_fill(buf, seed, counter_base=rank * n * size)
        pd = np.zeros(n, dtype=wga.PKT_DESC_DTYPE)
        pd["offset"] = np.arange(n, dtype=np.uint64) * size
        pd["len"] = size
        desc = torch.from_numpy(pd.view(np.uint8).copy()).to(dev)
        out = torch.empty(n, dtype=torch.uint16, device=dev)

        def launch():
            wga.checksum_desc(buf, desc, out=out)

        def sample(npk):
            k = min(n, npk)
            return buf[: k * size].cpu().numpy(), out[:k].cpu().numpy(), ("checksum", pd[:k].copy())

        cfg = {"workload": "config1: checksum(buf, 0) over 16,384 x 64 KiB random buffers per GPU "
                           "(tests/test-checksum.cpp:11-17 shape; BASELINE configs[0]), descriptor batch",
               "buffers_per_gpu": n, "buffer_bytes": size, "layout": "descriptor", "parallelism": f"shard{world}"}
        return Workload(launch, n, n * size, n * size + 2 * n + 16 * n, cfg, "weak", buf,
                        "wg::l4csum_coop_kernel<2,nt,4,4> (plain checksum, a 4-wave block per buffer: l4_coop)", rank * n, sample=sample,
                        counts=[n] * world,
                        metric="device-resident GiB/s, checksum(span, 0) over 64 KiB buffers (BASELINE config 1 shape)")
    if name in ("verify", "verify64d"):
        n = 1 << 20
        seed = 0x5EED00F1
        VSEG = SEG if name == "verify" else 64
        buf = torch.empty(n * VSEG, dtype=torch.uint8, device=dev)
        wga.synth_fill(buf, seed, counter_base=rank * n * VSEG)
        desc = wga.synth_desc_stride(n, VSEG, VSEG, 1, seed, rank * n, device=dev)  # mixed v4/v6 x TCP/UDP
        wga.synth_headers(buf, desc, seed, rank * n)
        wga.store_l4csum(buf, desc, wga.calc_l4_checksum_desc(buf, desc))  # received packets are valid
        torch.cuda.synchronize()
        verdict = torch.empty(n, dtype=torch.uint8, device=dev)
        l4 = torch.empty(n, dtype=torch.uint16, device=dev)

        def launch():
            wga.verify_desc(buf, desc, verdict=verdict, l4=l4)

        def post():
            # every packet must pass both gates; L4 results all zero
            flags = desc.view(torch.uint8).reshape(n, 16)[:, 14]
            okbits = 0x03
            bad = int(((verdict & okbits) != okbits).sum().item()) + int(torch.count_nonzero(l4.to(torch.int32)).item())
            v6 = int(((verdict & 0x10) != 0).sum().item())
            info = {"verify_failures": bad, "v6_packets": v6, "v6_expected": int((flags & 1).sum().item())}
            # small packets: the same batch shape with 64-B packets (valid,
            # mixed v4/v6 x TCP/UDP), wave-per-packet vs lane-per-descriptor
            # kernel (knob verify_small), bit-exact against each other
            b64 = torch.empty(n * 64, dtype=torch.uint8, device=dev)
            wga.synth_fill(b64, seed ^ 64)
            d64 = wga.synth_desc_stride(n, 64, 64, 1, seed, 0, device=dev)
            wga.synth_headers(b64, d64, seed, 0)
            wga.store_l4csum(b64, d64, wga.calc_l4_checksum_desc(b64, d64))
            v64 = torch.empty(n, dtype=torch.uint8, device=dev)
            l64 = torch.empty(n, dtype=torch.uint16, device=dev)
            saved = wga.tune_get("verify_small")
            small, ref = {}, None
            for kname, knob in (("wave_kernel", 0), ("default_auto", 7), ("compacting", 6), ("walking", 8)):
                wga.tune_set("verify_small", knob)
                for _ in range(10):
                    wga.verify_desc(b64, d64, verdict=v64, l4=l64)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(30):
                    wga.verify_desc(b64, d64, verdict=v64, l4=l64)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 30
                got = (v64.cpu().numpy(), l64.cpu().numpy())
                ref = got if ref is None else ref
                small[kname] = {"kernel_ms": round(ms, 5), "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
                                "GiB_s": round(n * 64 / (ms * 1e-3) / 2**30, 1),
                                "roofline_frac": round(n * (64 + 16 + 3) / (ms * 1e-3) / 8e12, 4),
                                "all_pass": bool(((got[0] & 3) == 3).all() and not got[1].any()),
                                "bit_exact_vs_wave_kernel": bool(np.array_equal(got[0], ref[0])
                                                                 and np.array_equal(got[1], ref[1]))}
            wga.tune_set("verify_small", saved)
            info["small_64B"] = {"packets": n, **small}
            del b64, d64, v64, l64
            return info

        def sample(npk):
            d = desc[:npk].cpu().numpy()
            v, l = wga.verify_desc(buf, desc[:npk])
            torch.cuda.synchronize()
            end = npk * VSEG
            return buf[:end].cpu().numpy(), (v.cpu().numpy(), l.cpu().numpy()), ("verify", d)

        cfg = {"workload": f"{name} (SURVEY §8 f1): 1,048,576 x {VSEG} B mixed IPv4/IPv6 x TCP/UDP per GPU, "
                           "checksums stored, evaluate_packet checksum gates (wg_verify_desc, default knobs)",
               "packets_per_gpu": n, "segment_size": VSEG, "layout": "descriptor", "parallelism": f"shard{world}"}
        kname = ("wg::verify_kernel<false> (verify_small=7 chose the wave kernel: no small packets sampled)"
                 if VSEG > 64 else "wg::verify_walk_kernel<true> (verify_small=7 chose the walking kernel, "
                 "consecutive layout: 64 of 64 sampled packets small)")
        return Workload(launch, n, n * VSEG, n * VSEG + 16 * n + n + 2 * n, cfg, "weak", buf,
                        kname, rank * n, sample=sample, counts=[n] * world, probe_run=VSEG,
                        metric="device-resident GiB/s, decap verify gates over packet batch (SURVEY f1)",
                        post=post)
    if name == "gro":
        n, slot = 1 << 22, 64
        rng = np.random.default_rng(0x5EED00F2 + rank)
        fam = rng.integers(0, 4, n)  # bit0 v6, bit1 tcp
        isv6, istcp = (fam & 1).astype(bool), (fam & 2).astype(bool)
        cs = np.where(isv6, 40, 20)
        hdr_len = cs + np.where(istcp, 20, 8)
        hdr = np.zeros((n, slot), dtype=np.uint8)
        # random addresses (v6: bytes 8-39; v4: 12-19), lengths/checksums stale (0)
        hdr[:, 8:40] = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        hdr[isv6, 0] = 0x60
        hdr[isv6, 6] = np.where(istcp[isv6], 6, 17)
        hdr[isv6, 7] = 64
        hdr[~isv6, 0:12] = np.array([0x45, 0, 0, 0, 0, 1, 0x40, 0, 64, 0, 0, 0], np.uint8)
        hdr[~isv6, 9] = np.where(istcp[~isv6], 6, 17)
        hdr[~isv6, 20:40] = 0
        gd = np.zeros(n, dtype=wga.GRO_DESC_DTYPE)
        gd["hdr_offset"] = np.arange(n, dtype=np.uint64) * slot
        gd["payload_bytes"] = rng.integers(1, 65000, n)
        gd["hdr_len"], gd["csum_start"] = hdr_len, cs
        gd["csum_offset"] = np.where(istcp, 16, 6)
        gd["flags"] = (isv6.astype(np.uint8)) | (istcp.astype(np.uint8) << 1)
        d_hdr = torch.from_numpy(hdr.reshape(-1)).to(dev)
        d_desc = torch.from_numpy(gd.view(np.uint8).copy()).to(dev)
        hdr_bytes = int(hdr_len.sum())
        written = int(np.where(isv6, 4, 6).sum() + 2 * (~istcp).sum())  # length fields, ip_sum, seed
        # Memory-side floor per flow (profiles/r02_store_granularity.json,
        # profiles/pmc_gro.json): the 24-B descriptor, the header chunks read
        # in 64-B memory blocks, the stores in 32-B sectors (the kernel's wide
        # stores: v4 bytes [0, 16), v6 [4, 8); UDP length + seed [cs+4, cs+8),
        # TCP seed [cs+16, cs+18)).
        ho = gd["hdr_offset"].astype(np.int64)
        need = np.where(isv6, 40, cs)
        c0 = ho & ~15
        c1 = c0 + 16 * (((ho & 15) + need - 1) // 16 + 1)
        rblk = (c1 - 1) // 64 - c0 // 64 + 1
        st_lo = np.where(isv6, ho + 4, ho)
        st_hi = np.where(isv6, ho + 8, ho + 16)
        f_lo = ho + cs + np.where(istcp, 16, 4)
        f_hi = f_lo + np.where(istcp, 2, 4)
        s1, s2 = st_lo // 32, (st_hi - 1) // 32
        t1, t2 = f_lo // 32, (f_hi - 1) // 32
        wsec = (s2 - s1 + 1) + (t2 - t1 + 1) - np.maximum(0, np.minimum(s2, t2) - np.maximum(s1, t1) + 1)
        phys = int(24 * n + 64 * rblk.sum() + 32 * wsec.sum())

        def launch():
            wga.gro_finalize(d_hdr, d_desc)

        def post():
            st = d_desc.cpu().numpy().view(wga.GRO_DESC_DTYPE)["status"]
            # self-check on the GPU: every finalized IPv4 header verifies to 0
            v4 = np.nonzero(~isv6)[0]
            pd = np.zeros(v4.size, dtype=wga.PKT_DESC_DTYPE)
            pd["offset"], pd["len"] = v4.astype(np.uint64) * slot, 20
            ipc = wga.checksum_desc(d_hdr, torch.from_numpy(pd.view(np.uint8).copy()).to(dev))
            return {"status_nonzero": int(np.count_nonzero(st)),
                    "ipv4_header_nonzero": int(torch.count_nonzero(ipc.to(torch.int32)).item())}

        def sample(npk):
            # the pre-finalize headers (host copy kept) and the GPU's finalized ones
            gd_s = gd[:npk].copy()
            got = d_hdr[: npk * slot].cpu().numpy()
            st = d_desc[: npk * 24].cpu().numpy().view(wga.GRO_DESC_DTYPE)["status"]
            return hdr.reshape(-1)[: npk * slot].copy(), (got, st), ("gro", gd_s)

        cfg = {"workload": "gro (SURVEY §8 f2): 4,194,304 coalesced flows per GPU, headers in 64 B slots, "
                           "mixed IPv4/IPv6 x TCP/UDP, in-place finalize (wg_gro_finalize)",
               "flows_per_gpu": n, "slot_bytes": slot, "parallelism": f"shard{world}"}
        cfg["alg_bytes_fields_only"] = n * 24 + hdr_bytes + written + n  # round 1-2 count: bytes the code touches
        cfg["alg_bytes_model"] = "24-B descriptor + header chunks in 64-B read blocks + stores in 32-B write sectors"
        return Workload(launch, n, n, phys, cfg, "weak", d_hdr,
                        "wg::gro_finalize_lds_kernel<true,5>", rank * n, sample=sample, counts=[n] * world,
                        metric="device-resident Mflows/s, GRO finalize (SURVEY f2)", unit="Mflows/s",
                        value_scale=1e-6, post=post)
    if name in ("verify64", "verify1500u"):
        return build_verify_uniform(wga, torch, rank, world, dev, 64 if name == "verify64" else 1504)
    if name == "config4small":
        return build_config4_small(wga, torch, rank, world, dev)
    if name == "config4strong":
        return build_config4_strong(wga, torch, rank, world, dev)
    if name == "encap_host":
        return build_encap_host(wga, torch, rank, world, dev)
    if name == "decap_host":
        return build_decap_host(wga, torch, rank, world, dev)
    # config4 bimodal
    n = 1 << 22
    seed = 0x5EED0004 + rank
    rng = np.random.default_rng(seed)
    lens = np.where(rng.random(n) < 0.5, 64, 9000).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])])
    total = int(offs[-1] + lens[-1])
    raw = np.zeros((n, 2), dtype=np.int64)
    raw[:, 0] = offs
    raw[:, 1] = lens | (20 << 32)  # len | csum_start << 32 | flags << 48 (v4/UDP)
    desc = torch.from_numpy(raw).to(dev)
    buf = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    wga.synth_fill(buf, seed)
    wga.synth_headers(buf, desc, seed, 0)
    out = torch.empty(n, dtype=torch.uint16, device=dev)

    def launch():
        wga.calc_l4_checksum_desc(buf, desc, out=out)

    def sample(npk):
        end = int(offs[npk - 1] + lens[npk - 1])
        return buf[:end].cpu().numpy(), out[:npk].cpu().numpy(), ("desc", raw[:npk])

    def post():
        """the small-only and large-only sub-batches
        (same buffer, the descriptors of one size class) and the whole batch,
        under the split-role kernel (default) and the wave-per-packet one
        (knob l4_small), timed like the main line (back-to-back launches
        between one event pair on the launch stream), each checked bit-exact
        against the main line's results."""
        sub = {}
        saved = wga.tune_get("l4_small")
        host_out = out.cpu().numpy()
        for name, size in (("small_64B", 64), ("large_9000B", 9000), ("mixed", None)):
            idx = np.nonzero(lens == size)[0] if size else np.arange(n)
            d_sub = torch.from_numpy(raw[idx]).to(dev)
            o_sub = torch.empty(len(idx), dtype=torch.uint16, device=dev)
            nbytes = int(lens[idx].sum())
            alg = nbytes + 18 * len(idx)  # bytes read + u16 written + 16-B descriptor
            for kname, small in (("wave_per_packet", 0), ("split_roles", 5)):
                wga.tune_set("l4_small", small)
                for _ in range(10):
                    wga.calc_l4_checksum_desc(buf, d_sub, out=o_sub)
                reps = 30
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(reps):
                    wga.calc_l4_checksum_desc(buf, d_sub, out=o_sub)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                same = bool(np.array_equal(o_sub.cpu().numpy(), host_out[idx]))
                sub.setdefault(name, {"packets": int(len(idx))})[kname] = {
                    "kernel_ms": round(ms, 5), "GiB_s": round(nbytes / (ms * 1e-3) / 2**30, 1),
                    "Mpps": round(len(idx) / (ms * 1e-3) / 1e6, 1),
                    "roofline_frac": round(alg / (ms * 1e-3) / 8e12, 4), "bit_exact_vs_main_line": same}
            del d_sub, o_sub
        wga.tune_set("l4_small", saved)
        # a uniform PacketBatch of 64-B segments (same packet count as the
        # 64-B sub-batch): the small-packet kernel is chosen from segment_size
        n64 = int((lens == 64).sum())
        b64 = torch.empty(n64 * 64, dtype=torch.uint8, device=dev)
        wga.synth_fill(b64, seed ^ 64)
        wga.synth_headers(b64, wga.synth_desc_stride(n64, 64, 64, 0, seed, 0, device=dev), seed, 0)
        o64 = torch.empty(n64, dtype=torch.uint16, device=dev)
        su = wga.tune_get("l4_small_uniform")
        res = {}
        ref = None
        nt0 = wga.tune_get("l4_nt")
        for kname, knob, nt in (("wave_per_packet", 0, nt0), ("small_kernel_lane", 2, nt0)):
            wga.tune_set("l4_small_uniform", knob)
            wga.tune_set("l4_nt", nt)
            for _ in range(10):
                wga.calc_l4_checksum_batch(b64, 64, False, False, 20, out=o64)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(30):
                wga.calc_l4_checksum_batch(b64, 64, False, False, 20, out=o64)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 30
            got = o64.cpu().numpy()
            ref = got if ref is None else ref
            res[kname] = {"kernel_ms": round(ms, 5), "GiB_s": round(n64 * 64 / (ms * 1e-3) / 2**30, 1),
                          "Mpps": round(n64 / (ms * 1e-3) / 1e6, 1),
                          "roofline_frac": round(n64 * 66 / (ms * 1e-3) / 8e12, 4),
                          "bit_exact_vs_wave_kernel": bool(np.array_equal(got, ref))}
        wga.tune_set("l4_small_uniform", su)
        wga.tune_set("l4_nt", nt0)
        sub["uniform_64B"] = {"packets": n64, **res}
        del b64, o64
        return {"sub_batches": sub}

    cfg = {"workload": "config4: 4,194,304 IPv4/UDP packets, 64 B / 9000 B 50/50, packed, descriptor batch",
           "packets_per_gpu": n, "layout": "descriptor", "parallelism": f"shard{world}"}
    return Workload(launch, n, total, total + 2 * n + 16 * n, cfg, "weak", buf, "wg::l4csum_split_kernel<1,nt> (l4_small=5)",
                    rank * n, out, desc, sample, [n] * world, post=post)


def config4_lengths():
    """BASELINE config 4's packet lengths: 4,194,304 packets, 64 B or 9000 B
    50/50 by a seeded draw (0x5EED0004), packed back to back."""
    import numpy as np

    n = 1 << 22
    rng = np.random.default_rng(0x5EED0004)
    lens = np.where(rng.random(n) < 0.5, 64, 9000).astype(np.int64)
    return lens, np.concatenate([[0], np.cumsum(lens[:-1])])


def build_config4_strong(wga, torch, rank: int, world: int, dev) -> Workload:
    """Config 4's ONE 4 M-packet bimodal batch split across the ranks by BYTES
    (dist.shard_bounds_by_bytes): rank r holds the packets of
    its byte-balanced range, generated from the global byte counter and packet
    index, so its shard equals the same slice of the N = 1 batch and the
    all-reduced result hash is the same at every N."""
    import numpy as np

    from wireglider_amd import dist as wdist

    seed = 0x5EED0004
    lens, offs = config4_lengths()
    bounds = wdist.shard_bounds_by_bytes(lens, world)
    lo, hi = bounds[rank]
    n = hi - lo
    g0 = int(offs[lo]) if n else 0
    base = g0 & ~15  # synth_fill's counter base is 16-B aligned: start the shard buffer there
    end = int(offs[hi - 1] + lens[hi - 1]) if n else base
    raw = np.zeros((max(n, 1), 2), dtype=np.int64)
    raw[:n, 0] = offs[lo:hi] - base
    raw[:n, 1] = lens[lo:hi] | (20 << 32)  # v4/UDP, csum_start 20
    desc = torch.from_numpy(raw[:n].copy()).to(dev)
    buf = torch.empty(end - base + 16, dtype=torch.uint8, device=dev)
    wga.synth_fill(buf, seed, counter_base=base)
    wga.synth_headers(buf, desc, seed, lo)
    out = torch.empty(max(n, 1), dtype=torch.uint16, device=dev)[:n]

    def launch():
        wga.calc_l4_checksum_desc(buf, desc, out=out)

    payload = int(lens[lo:hi].sum())
    counts = [b - a for a, b in bounds]
    cfg = {"workload": "config4 strong: ONE 4,194,304-packet 64 B / 9000 B IPv4/UDP batch split across the GPUs "
                       "by bytes (shard_bounds_by_bytes)", "packets_total": int(lens.size), "packets_per_gpu": n,
           "layout": "descriptor", "parallelism": f"shard{world} (byte-balanced contiguous ranges)"}
    return Workload(launch, n, payload, payload + 18 * n, cfg, "strong", buf,
                    "wg::l4csum_split_kernel<1,nt> (l4_small=5)", lo, out, desc, None, counts)


def build_config4_small(wga, torch, rank: int, world: int, dev) -> Workload:
    """Config 4's 64-B sub-batch as a workload of its own, so
    PMC and kernel stats cover it: the 2,098,300 64-B packets of config 4's
    batch, where they lie between the 9000-B ones (8-B aligned), through
    the default descriptor kernel.  The physical floor is counted beside
    the algorithmic bytes: each packet touches one or two 64-B memory blocks."""
    import numpy as np

    seed = 0x5EED0004
    lens, offs = config4_lengths()
    idx = np.nonzero(lens == 64)[0]
    raw = np.zeros((idx.size, 2), dtype=np.int64)
    raw[:, 0] = offs[idx]
    raw[:, 1] = 64 | (20 << 32)
    total = int(offs[-1] + lens[-1])
    buf = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    wga.synth_fill(buf, seed)
    full = np.zeros((lens.size, 2), dtype=np.int64)
    full[:, 0] = offs
    full[:, 1] = lens | (20 << 32)
    wga.synth_headers(buf, torch.from_numpy(full).to(dev), seed, 0)
    desc = torch.from_numpy(raw).to(dev)
    n = idx.size
    out = torch.empty(n, dtype=torch.uint16, device=dev)

    def launch():
        wga.calc_l4_checksum_desc(buf, desc, out=out)

    def sample(npk):
        k = min(n, npk)
        end = int(raw[k - 1, 0]) + 64
        return buf[:end].cpu().numpy(), out[:k].cpu().numpy(), ("desc", raw[:k])

    o = offs[idx]
    blocks = ((o + 63) // 64 - o // 64 + 1)
    phys = int(64 * blocks.sum()) + 18 * n
    cfg = {"workload": "config4small: config 4's 64-B sub-batch (2,098,300 IPv4/UDP packets between its 9000-B ones, "
                       "8-B aligned), descriptor batch", "packets_per_gpu": int(n), "layout": "descriptor",
           "physical_floor_bytes": phys,
           "physical_floor_model": "64-B memory blocks touched by each packet (1 or 2) + 16-B descriptor + 2-B result",
           "parallelism": f"shard{world}"}
    return Workload(launch, n, 64 * n, 82 * n, cfg, "weak", buf, "wg::l4csum_split_kernel<1,nt> (l4_small=5)", 0,
                    out, desc, sample, [n] * world)


def build_verify_uniform(wga, torch, rank: int, world: int, dev, seg: int) -> Workload:
    """SURVEY §8 f1 on the decap worker's own batch shape: the plaintexts of
    one UDP GRO batch are a uniform PacketBatch (worker/decap.cpp:145-151,
    worker/decap_ref.cpp:78-86), verified by wg_verify_uniform — 1,048,576
    valid IPv4/IPv6 x TCP/UDP packets of `seg` bytes (64: TCP ACK-sized
    batches, a lane per packet; 1504: full-size, a wave per packet)."""
    import numpy as np

    n, seed = 1 << 20, 0x5EED00F3 + seg
    buf = torch.empty(n * seg, dtype=torch.uint8, device=dev)
    wga.synth_fill(buf, seed, counter_base=rank * n * seg)
    desc = wga.synth_desc_stride(n, seg, seg, 1, seed, rank * n, device=dev)  # mixed v4/v6 x TCP/UDP
    wga.synth_headers(buf, desc, seed, rank * n)
    wga.store_l4csum(buf, desc, wga.calc_l4_checksum_desc(buf, desc))
    torch.cuda.synchronize()
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    l4 = torch.empty(n, dtype=torch.uint16, device=dev)

    def launch():
        wga.verify_uniform(buf, seg, verdict=verdict, l4=l4)

    def post():
        bad = int(((verdict & 3) != 3).sum().item()) + int(torch.count_nonzero(l4.to(torch.int32)).item())
        # the same packets through the descriptor entry (its default kernel), bit-exact
        v2, l2 = wga.verify_desc(buf, desc)
        torch.cuda.synchronize()
        return {"verify_failures": bad, "equal_to_wg_verify_desc": bool(torch.equal(v2, verdict) and torch.equal(l2, l4))}

    def sample(npk):
        d = desc[:npk].cpu().numpy()
        v, l = wga.verify_uniform(buf[: npk * seg], seg)
        torch.cuda.synchronize()
        return buf[: npk * seg].cpu().numpy(), (v.cpu().numpy(), l.cpu().numpy()), ("verify", d)

    kern = "wg::verify_uniform_lane_kernel (a lane per packet)" if seg <= 64 else "wg::verify_kernel<4,8,0,true,true>"
    cfg = {"workload": f"verify{'64' if seg <= 64 else '1500u'} (SURVEY §8 f1): 1,048,576 x {seg} B mixed IPv4/IPv6 x "
                       "TCP/UDP per GPU, checksums stored, a uniform PacketBatch (one GRO batch's plaintexts) through "
                       "wg_verify_uniform", "packets_per_gpu": n, "segment_size": seg, "layout": "uniform",
           "parallelism": f"shard{world}"}
    return Workload(launch, n, n * seg, n * (seg + 3), cfg, "weak", buf, kern, rank * n, sample=sample,
                    counts=[n] * world, post=post, probe_run=seg if seg <= 2048 else 0,
                    metric="device-resident GiB/s, decap verify gates over a uniform packet batch (SURVEY f1)")


def _pinned_copy(wga, t):
    """A device tensor's bytes in a wg_host_alloc (pinned) buffer."""
    import numpy as np

    pb = wga.PinnedBuffer(t.numel())
    pb.array[:] = t.cpu().numpy().reshape(-1)
    return pb


def pcie_ceiling(torch, h2d_bytes: int, d2h_bytes: int, reps: int = 5) -> dict:
    """Raw PCIe copy rates on this box with pinned host memory: hipMemcpyAsync
    H2D alone, D2H alone, and both at once on two streams (PCIe is full
    duplex) — the ceiling of a host-memory pipeline moving these bytes."""
    dev = torch.device("cuda", torch.cuda.current_device())
    hin = torch.empty(h2d_bytes, dtype=torch.uint8).pin_memory()
    hout = torch.empty(d2h_bytes, dtype=torch.uint8).pin_memory()
    din = torch.empty(h2d_bytes, dtype=torch.uint8, device=dev)
    dout = torch.empty(d2h_bytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def run(up, down):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            if up:
                with torch.cuda.stream(s1):
                    din.copy_(hin, non_blocking=True)
            if down:
                with torch.cuda.stream(s2):
                    hout.copy_(dout, non_blocking=True)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    run(True, True)
    t_up, t_down, t_both = run(True, False), run(False, True), run(True, True)
    res = {"h2d_GBps": round(h2d_bytes / t_up / 1e9, 2), "d2h_GBps": round(d2h_bytes / t_down / 1e9, 2),
           "both_GBps": round((h2d_bytes + d2h_bytes) / t_both / 1e9, 2),
           "both_ms": round(t_both * 1e3, 3), "bytes": {"h2d": h2d_bytes, "d2h": d2h_bytes}}
    del hin, hout, din, dout
    return res


def build_encap_host(wga, torch, rank: int, world: int, dev) -> Workload:
    """The encap worker's step from host memory (SURVEY §8 f3 with A6 + f4,
    worker/encap.cpp:22-170): 32,768 tun reads of config 3's shape (64 KiB
    IPv4/TCP super-buffers, 1,460-B segments) in a pinned buffer ->
    wg_encap_host (chunked H2D, the headers-only GSO split + encryption of
    every segment on the device, messages D2H into a pinned send buffer).
    value = GiB/s of tun input, host memory to host memory."""
    import numpy as np

    n, in_stride, in_len, hdr, gso, seed = 1 << 15, 65536, 65535, 40, 1460, 0x5EED00E6
    seg = hdr + gso
    nseg = (in_len - hdr + gso - 1) // gso
    out_len = in_len - hdr + nseg * hdr
    mstride = wga.aead_message_stride(seg)
    mbytes = (nseg - 1) * mstride + wga.aead_message_stride(out_len - (nseg - 1) * seg)
    mcap = nseg * mstride
    d_in = torch.empty(n * in_stride, dtype=torch.uint8, device=dev)
    wga.synth_fill(d_in, seed, counter_base=rank * n * in_stride)
    pd = np.zeros(n, dtype=wga.PKT_DESC_DTYPE)
    pd["offset"] = np.arange(n, dtype=np.uint64) * in_stride
    pd["len"], pd["csum_start"], pd["flags"] = in_len, 20, 2
    wga.synth_headers(d_in, torch.from_numpy(pd.view(np.uint8).copy()).to(dev), seed, rank * n)
    gd = np.zeros(n, dtype=wga.GSO_DESC_DTYPE)
    gd["in_offset"] = pd["offset"]
    gd["in_len"], gd["out_cap"] = in_len, 73216  # the reference's per-worker outbuf (worker/encap.cpp:26)
    gd["vnet"]["flags"], gd["vnet"]["gso_type"], gd["vnet"]["gso_size"] = 1, 1, gso
    gd["vnet"]["csum_start"], gd["vnet"]["csum_offset"] = 20, 16
    pin_in = _pinned_copy(wga, d_in)
    pin_out = wga.PinnedBuffer(n * mcap)
    key = np.random.default_rng(seed).integers(0, 256, 32, dtype=np.uint8).tobytes()
    rx, c0 = 0x0E0CAA, 1 + rank * n * nseg
    state = {}

    def launch():
        state["r"] = wga.encap_host(pin_in.array, gd, key, rx, c0, nseg, seg, mcap, msgs=pin_out.array)

    def post():
        _, res, gres, nxt = state["r"]
        ok = bool(np.all(res["nmsg"] == nseg) and np.all(res["msg_bytes"] == mbytes)
                  and np.array_equal(res["counter0"], c0 + np.arange(n, dtype=np.uint64) * nseg)
                  and np.all(gres["status"] == 0))
        # a sample decrypted back on the device and compared with the split's segments
        k = 256
        full = torch.from_numpy(np.concatenate([pin_out.array[i * mcap: i * mcap + (nseg - 1) * mstride]
                                                for i in range(k)])).to(dev)
        pt, st = wga.aead_decrypt_batch(full, mstride, key)
        ref = torch.empty(k * 73216, dtype=torch.uint8, device=dev)
        gdk = gd[:k].copy()
        gdk["out_offset"] = np.arange(k, dtype=np.uint64) * 73216
        wga.gso_split(d_in[: k * in_stride].clone(), torch.from_numpy(gdk.view(np.uint8).copy()).to(dev), ref)
        segs = torch.cat([ref[i * 73216: i * 73216 + (nseg - 1) * seg] for i in range(k)])
        torch.cuda.synchronize()
        same = bool(torch.equal(pt.view(-1, mstride - 32)[:, :seg].reshape(-1), segs))
        return {"results_ok": ok, "next_counter": int(nxt), "next_counter_expected": int(c0 + n * nseg),
                "sample_super_buffers_decrypted": k, "sample_plaintexts_equal_segments": same,
                "sample_status_nonzero": int(torch.count_nonzero(st).item())}

    def sample(_npk):
        k = min(n, 1024)
        gk = gd[:k].copy()
        gk["out_offset"] = np.arange(k, dtype=np.uint64) * 73216
        return (pin_in.array[: k * in_stride].copy(), pin_out.array[: k * mcap].copy(),
                ("encap", gk, k * 73216, key, rx, c0, seg, nseg, mcap, mbytes))

    cfg = {"workload": "encap_host: 32,768 tun reads of 64 KiB IPv4/TCP (config 3 shape) in pinned host memory -> "
                       "wg_encap_host (H2D, GSO split + ChaCha20-Poly1305 per 1460-B segment, messages D2H to pinned "
                       "memory), one peer", "super_buffers_per_gpu": n, "segments_per_buffer": nseg,
           "message_stride": mstride, "parallelism": f"shard{world}", "entry": "wg_encap_host",
           "host_chunk_mb": wga.tune_get("host_chunk_mb")}
    return Workload(launch, n, n * in_len, n * (in_len + mbytes), cfg, "weak", d_in,
                    "wg_encap_host pipeline (H2D / wg_encap_batch kernels / D2H on three streams)", rank * n,
                    sample=sample, counts=[n] * world, post=post,
                    metric="host-memory GiB/s of tun input, encap step incl. PCIe (SURVEY f3 + A6 + f4)",
                    pcie={"h2d": n * in_stride, "d2h": n * mcap})


def build_decap_host(wga, torch, rank: int, world: int, dev) -> Workload:
    """The decap worker's step from host memory (SURVEY §8 f3 with f4 + f1,
    worker/decap.cpp:90-156 -> worker/decap_ref.cpp:53-89): a UDP GRO batch
    of 1,048,576 data messages (1,504-B inner IPv4/IPv6 x TCP/UDP packets, a
    multiple of 16 so every gate runs) in a pinned buffer -> wg_decap_host
    (chunked H2D, decrypt + verify gates fused on the device, plaintext and
    verdicts D2H into pinned memory).  value = GiB/s of UDP messages."""
    import numpy as np

    n, s2, seed = 1 << 20, 1504, 0x5EED00D4
    m2 = wga.aead_message_stride(s2)
    pk = torch.empty(n * s2, dtype=torch.uint8, device=dev)
    wga.synth_fill(pk, seed, counter_base=rank * n * s2)
    d2 = wga.synth_desc_stride(n, s2, s2, 1, seed, rank * n, device=dev)
    wga.synth_headers(pk, d2, seed, rank * n)
    wga.store_l4csum(pk, d2, wga.calc_l4_checksum_desc(pk, d2))
    key = np.random.default_rng(seed).integers(0, 256, 32, dtype=np.uint8).tobytes()
    msgs, _ = wga.aead_encrypt_batch(pk, s2, key, 0x1D, 77 + rank * n)
    torch.cuda.synchronize()
    pin_m = _pinned_copy(wga, msgs[: n * m2])
    del msgs
    pin_p = wga.PinnedBuffer(n * s2)
    state = {}

    def launch():
        state["r"] = wga.decap_host(pin_m.array, m2, key, verify=True, plain=pin_p.array)

    def post():
        _, st, ver, l4 = state["r"]
        same = bool(torch.equal(torch.from_numpy(pin_p.array).to(dev), pk))
        return {"status_nonzero": int(np.count_nonzero(st)), "verify_failures": int(np.count_nonzero((ver & 3) != 3)),
                "l4_nonzero": int(np.count_nonzero(l4)), "plaintext_equal_packets": same}

    def sample(_npk):
        k = 1 << 16
        _, st, ver, l4 = state["r"] if "r" in state else wga.decap_host(pin_m.array, m2, key, plain=pin_p.array)
        return (None, (st[:k].copy(), ver[:k].copy(), l4[:k].copy()),
                ("decap", key, m2, pin_m.array[: k * m2].copy()))

    cfg = {"workload": "decap_host: a UDP GRO batch of 1,048,576 WireGuard data messages (1,504-B inner IPv4/IPv6 x "
                       "TCP/UDP packets) in pinned host memory -> wg_decap_host (H2D, decrypt + verify gates fused, "
                       "plaintext + verdicts D2H to pinned memory)", "messages_per_gpu": n, "message_stride": m2,
           "parallelism": f"shard{world}", "entry": "wg_decap_host", "host_chunk_mb": wga.tune_get("host_chunk_mb")}
    return Workload(launch, n, n * m2, n * (m2 + s2 + 4), cfg, "weak", pk,
                    "wg_decap_host pipeline (H2D / aead_kernel<..,dec,verify> / D2H on three streams)", rank * n,
                    sample=sample, counts=[n] * world, post=post,
                    metric="host-memory GiB/s of UDP data messages, decap step incl. PCIe (SURVEY f3 + f4 + f1)",
                    pcie={"h2d": n * m2, "d2h": n * (s2 + 4)})


def build_encap(wga, torch, rank: int, world: int, dev, fused: bool = True) -> Workload:
    """The encap worker's data path on the device (worker/encap.cpp:107-160):
    config 3's 262,144 x 64 KiB tun super-buffers -> do_tun_gso_split ->
    Peer::encrypt for every segment in order with encrypt_nonce++, one peer,
    no host round trip.  fused: one wg_encap_batch per step (headers-only
    split, payload encrypted from the input); else wg_gso_split +
    wg_encap_encrypt (workload encap_2call).  value = GiB/s of tun input."""
    import numpy as np

    n, in_stride, out_stride, in_len = 1 << 18, 65536, 73216, 65535
    hdr, gso, seed = 40, 1460, 0x5EED00E5
    seg = hdr + gso
    nseg = (in_len - hdr + gso - 1) // gso
    out_len = in_len - hdr + nseg * hdr
    mstride = wga.aead_message_stride(seg)
    last = out_len - (nseg - 1) * seg
    mbytes = (nseg - 1) * mstride + wga.aead_message_stride(last)
    buf = torch.empty(n * in_stride, dtype=torch.uint8, device=dev)
    wga.synth_fill(buf, seed, counter_base=rank * n * in_stride)
    pd = np.zeros(n, dtype=wga.PKT_DESC_DTYPE)
    pd["offset"] = np.arange(n, dtype=np.uint64) * in_stride
    pd["len"], pd["csum_start"], pd["flags"] = in_len, 20, 2
    wga.synth_headers(buf, torch.from_numpy(pd.view(np.uint8).copy()).to(dev), seed, rank * n)
    gd = np.zeros(n, dtype=wga.GSO_DESC_DTYPE)
    gd["in_offset"] = pd["offset"]
    gd["out_offset"] = np.arange(n, dtype=np.uint64) * out_stride
    gd["in_len"], gd["out_cap"] = in_len, out_stride
    gd["vnet"]["flags"], gd["vnet"]["gso_type"], gd["vnet"]["gso_size"] = 1, 1, gso
    gd["vnet"]["csum_start"], gd["vnet"]["csum_offset"] = 20, 16
    d_desc = torch.from_numpy(gd.view(np.uint8).copy()).to(dev)
    outb = torch.empty(n * out_stride, dtype=torch.uint8, device=dev)
    res = torch.empty(n * wga.GSO_RESULT_BYTES, dtype=torch.uint8, device=dev)
    mcap = nseg * mstride
    msg_off_np = np.arange(n, dtype=np.int64) * mcap
    msg_off = torch.from_numpy(msg_off_np).to(dev)
    msgs = torch.empty(n * mcap, dtype=torch.uint8, device=dev)
    eres = torch.zeros(n * wga.ENCAP_RESULT_BYTES, dtype=torch.uint8, device=dev)
    work = torch.empty(n + 1024, dtype=torch.int32, device=dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    key = np.random.default_rng(seed).integers(0, 256, 32, dtype=np.uint8).tobytes()
    rx, c0 = 0x0E0CA9, 1 + rank * n * nseg

    def launch():
        if fused:
            wga.encap_batch(buf, d_desc, outb, res, key, rx, c0, msg_off, mcap, nseg, seg, msgs, results=eres,
                            work=work, total=tot)
        else:
            wga.gso_split(buf, d_desc, outb, results=res)
            wga.encap_encrypt(buf, outb, d_desc, res, key, rx, c0, msg_off, mcap, nseg, seg, msgs, results=eres,
                              work=work, total=tot)

    def post():
        # every super-buffer: 45 messages at consecutive counters, and a
        # sample of them decrypted back to their GSO segments on the device
        e = eres.cpu().numpy().view(wga.ENCAP_RESULT_DTYPE)
        ok = bool(np.all(e["nmsg"] == nseg) and np.all(e["msg_bytes"] == mbytes)
                  and np.array_equal(e["counter0"], c0 + np.arange(n, dtype=np.uint64) * nseg))
        k = 256
        full = torch.cat([msgs[int(msg_off_np[i]): int(msg_off_np[i]) + (nseg - 1) * mstride] for i in range(k)])
        pt, st = wga.aead_decrypt_batch(full, mstride, key)
        # the reference segments: a full split of the sample (the fused call
        # leaves only the headers in outb; splitting again is idempotent)
        ref = torch.empty(k * out_stride, dtype=torch.uint8, device=dev)
        wga.gso_split(buf[: k * in_stride], d_desc[: k * wga.GSO_DESC_BYTES], ref)
        segs = torch.cat([ref[i * out_stride: i * out_stride + (nseg - 1) * seg] for i in range(k)])
        torch.cuda.synchronize()
        same = bool(torch.equal(pt.view(-1, mstride - 32)[:, :seg].reshape(-1), segs))
        return {"results_ok": ok, "messages_total": int(tot.cpu()[0]), "sample_super_buffers_decrypted": k,
                "sample_plaintexts_equal_segments": same, "sample_status_nonzero": int(torch.count_nonzero(st).item())}

    def sample(_npk):
        k = min(n, 1024)
        return (buf[: k * in_stride].cpu().numpy(), msgs[: k * mcap].cpu().numpy(),
                ("encap", gd[:k].copy(), k * out_stride, key, rx, c0, seg, nseg, mcap, mbytes))

    cfg = {"workload": "encap: config 3's 262,144 x 64 KiB IPv4/TCP tun super-buffers -> do_tun_gso_split (45 x "
                       "1460 B segments) -> Peer::encrypt per segment, one peer, consecutive counters (the encap "
                       "worker, worker/encap.cpp:107-160)", "super_buffers_per_gpu": n, "segments_per_buffer": nseg,
           "message_stride": mstride, "parallelism": f"shard{world}",
           "entry": "wg_encap_batch" if fused else "wg_gso_split + wg_encap_encrypt"}
    # the split reads the input and writes the segments (fused: only each
    # segment's header block, pad64(hdr) bytes); the AEAD reads every
    # segment's plaintext once and writes the messages (synthesis: the AEAD
    # is the only reader of the input and writes the header blocks itself)
    split_w = n * nseg * ((hdr + 63) // 64 * 64) if fused else n * out_len
    aead_k = aead_kernel_symbol(wga, seg, gso=2 if fused else 1)
    # with header synthesis (the AEAD builds the headers while it encrypts)
    # the input is read once: no separate pass of the segments
    synth = fused and "true>(" in aead_k
    alg = (n * in_len + split_w + n * (wga.GSO_DESC_BYTES + wga.GSO_RESULT_BYTES)
           + (0 if synth else n * out_len) + n * mbytes + n * (wga.ENCAP_RESULT_BYTES + 8))
    return Workload(launch, n, n * in_len, alg, cfg, "weak", buf,
                    ("wg_encap_batch (plan + finalize kernels, the headers-only split walking the list of "
                     "super-buffers left to it (none here: the AEAD synthesizes every segment header), "
                     "2 scan kernels + %s)" if fused and "true>(" in aead_k else
                     "wg_encap_batch (3 split kernels, headers only, + 2 scan kernels + %s)" if fused else
                     "wg_gso_split (3 kernels) + wg_encap_encrypt (2 scan kernels + %s)") % aead_k,
                    rank * n, sample=sample, counts=[n] * world, post=post, copy_dst=msgs,
                    valu_kernel=aead_k if synth else None,
                    metric="device-resident GiB/s of tun input, GSO split + data-message encryption (encap worker)")


def settle(torch, fn, seconds: float) -> int:
    """Run `fn` back to back until `seconds` of wall time have passed, so the
    timed region starts at the sustained clock/memory state rather than the
    idle ramp (MI355X: the first ~10 launches run up to 30% slower)."""
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < seconds:
        for _ in range(20):
            fn()
        k += 20
        torch.cuda.synchronize()
    return k


def measured_read_peak(torch, wga, buf, iters: int = 30, run_bytes: int = 0) -> dict:
    """Read probe over the batch buffer itself: the same bytes, read with no
    checksum work (GB/s) — contiguous one-shot waves of 2/4/8 KiB, and, for
    batches of <= 2 KiB packets (run_bytes), the L4 kernel's own issue
    structure (4 packets per wave, two 16-B loads per lane each).  The best of
    them is the line's read_probe_reference: a reference point for the
    kernel, not a ceiling (the L4 kernel has measured 0.8 % above it)."""
    # The WHOLE buffer, in <= 4 GiB slices: a 25 GB buffer's rate depends on
    # its physical pages (profiles/r02_config5_placement.json), so the
    # ceiling must read the same pages the kernel reads.
    acc = torch.zeros(1, dtype=torch.int64, device=buf.device)
    variants = [(f"contiguous_{k}KiB", k, 0) for k in (2, 4, 8)]
    if 0 < run_bytes <= 2048:
        variants.append((f"runs_{run_bytes}B_x4_per_wave", 1, run_bytes))
    iters = iters if buf.numel() <= 4 << 30 else max(3, iters * (4 << 30) // buf.numel())
    rates = {}
    # best of 3 interleaved passes per variant: a ceiling, not a sample
    for _ in range(3):
        for name, kib, run in variants:
            step = (4 << 30) // (16 * run) * 16 * run if run else 4 << 30  # slices stay 16-B aligned
            views = [buf[o: o + min(step, buf.numel() - o) // 16 * 16] for o in range(0, buf.numel(), step)]
            views = [v for v in views if v.numel() >= max(run, 16)]
            nb = sum(v.numel() // run * run if run else v.numel() for v in views)

            def once():
                for v in views:
                    wga.probe_read(v, acc, kib, run_bytes=run)

            settle(torch, once, 0.05)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                once()
            e1.record()
            torch.cuda.synchronize()
            rates[name] = max(rates.get(name, 0.0), round(nb * iters / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1))
    return {"best": max(rates.values()), "variants": rates, "bytes": int(buf.numel())}


def measured_copy_peak(torch, wga, src, dst, iters: int = 3) -> dict:
    """Copy-roofline probe over the workload's own buffers, in the same run:
    dst = src over min(len) bytes by one-shot waves (wg_probe_copy), non-temporal
    and default-policy loads / stores at 1 / 2 / 4 KiB per wave; best of 3
    interleaved passes per variant.  Rate = bytes read + bytes written per
    second, the unit of a read+write kernel's `achieved`.  Overwrites dst."""
    n = min(src.numel(), dst.numel()) // 16 * 16
    s, d = src[:n], dst[:n]
    variants = [(f"{pol}_{k}KiB", k, pol == "default") for pol in ("nt", "default") for k in (1, 2, 4)]
    rates = {}
    for _ in range(3):
        for name, kib, dflt in variants:
            wga.probe_copy(s, d, kib, default_policy=dflt)  # warm-up launch
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                wga.probe_copy(s, d, kib, default_policy=dflt)
            e1.record()
            torch.cuda.synchronize()
            rates[name] = max(rates.get(name, 0.0), round(2 * n * iters / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1))
    return {"best": max(rates.values()), "variants": rates, "bytes_each_way": int(n)}


def wga_stride(seg: int) -> int:
    """Peer::expected_encrypt_size (include/proto/proto.hpp:266-269)."""
    return 16 + (seg + 15) // 16 * 16 + 16


def _rep_rates(fn, units: float, seconds: float, reps: int, before=None, after=None) -> list:
    """`reps` repetitions, each running fn() back to back until `seconds` of
    wall time have passed (before() ahead of each and after() behind each,
    untimed); the rate (units per second) of each repetition."""
    out = []
    for _ in range(reps):
        if before is not None:
            before()
        k, t0 = 0, time.perf_counter()
        while True:
            fn()
            k += 1
            t = time.perf_counter() - t0
            if t >= seconds:
                break
        out.append(units * k / t)
        if after is not None:
            after()
    return out


def _cpu_freqs_khz(cpus) -> list | None:
    """scaling_cur_freq (kHz) of each CPU, or None where the host does not
    expose it (read right after a repetition: the clock the pinned worker ran
    at, to within the governor's sampling)."""
    out = []
    for c in cpus:
        try:
            out.append(int(Path(f"/sys/devices/system/cpu/cpu{c}/cpufreq/scaling_cur_freq").read_text()))
        except Exception:
            out.append(None)
    return out if any(x is not None for x in out) else None


def _spread(rates: list, scale: float) -> dict:
    """Median / min / max of the repetitions after the first (dropped: first
    touch of the pages, thread start-up); every value is kept in the line.
    spread_pct = the largest deviation from the median with the single most
    deviant repetition set aside (on this shared host one repetition in 7-8
    now and then lands on a neighbour's burst: 56 vs 77 GiB/s); spread_pct_all
    counts every repetition."""
    vals = [x * scale for x in rates]
    r = sorted(vals[1:] if len(vals) > 1 else vals)
    med = r[len(r) // 2] if len(r) % 2 else 0.5 * (r[len(r) // 2 - 1] + r[len(r) // 2])
    dev = lambda xs: round(100.0 * max(abs(x - med) for x in xs) / med, 2) if med and xs else None  # noqa: E731
    trimmed = sorted(r, key=lambda x: abs(x - med))[:-1] if len(r) >= 5 else r
    return {"median": med, "min": r[0], "max": r[-1], "reps": len(r),
            "spread_pct": dev(trimmed), "spread_pct_all": dev(r), "spread_set_aside": len(r) - len(trimmed),
            "values": [round(v, 3) for v in vals], "dropped_first": len(vals) > 1}


def _read_probe_rate(oracle, buf, threads: int, seconds: float = 1.0) -> dict:
    """GiB/s of a read-only pass (64-bit word sums, oracle.read_probe) over
    the CPU sample's own buffer on the current leg's pinned workers: the
    memory path those CPUs get with no checksum work.  One untimed pass, then
    passes until `seconds` have run; best of 3 such runs."""
    oracle.read_probe(buf, threads)
    best = 0.0
    for _ in range(3):
        k, t0 = 0, time.perf_counter()
        while True:
            oracle.read_probe(buf, threads)
            k += 1
            t = time.perf_counter() - t0
            if t >= seconds / 3:
                break
        best = max(best, buf.size // 4096 * 4096 * k / t)
    return {"GiB_s": round(best * 2.0**-30, 3), "threads": threads, "bytes": int(buf.size)}


def oracle_numa(c):
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only

    return oracle.numa_of(c)


def _placement_evidence(quiet, cpus_all, workers, nbytes, scale, unit, all_s, one_s, read_all, read_one,
                        buf) -> dict:
    """where the all-core leg's CPUs sit (L3
    domains), each worker's own rate (its equal share of the sample's bytes
    over its busy time in the pool), and whether the leg is bound by the
    memory path of those CPUs (its rate against a read-only probe over the
    same buffer on the same CPUs) or by the checksum work."""
    out = {"l3_domains": quiet.get("l3_domains") if quiet else None}
    if workers:
        share = nbytes / len(workers)
        rates = [round(share * c / b * scale, 3) if b > 0 else None for b, c in workers]
        good = [r for r in rates if r]
        out["per_worker"] = {
            "cpus": cpus_all, "numa_node": [oracle_numa(c) for c in cpus_all] if cpus_all else None,
            "rate": rates, "unit": unit, "busy_s": [round(b, 3) for b, _ in workers],
            "calls": [c for _, c in workers],
            "min_over_max": round(min(good) / max(good), 4) if good else None,
            "note": "worker t's equal share of the sample's bytes per call x its calls / its own busy time in "
                    "the pool (orc_pool_stats), over the timed repetitions"}
    if read_all and read_one and unit == "GiB/s":
        ra, ro = read_all["GiB_s"], read_one["GiB_s"]
        ca, co = all_s["median"], one_s["median"]
        frac = ca / ra if ra else None
        out["read_probe"] = {"all": read_all, "one": read_one, "scaling_all_over_one": round(ra / ro, 3) if ro else None,
                             "checksum_scaling_all_over_one": round(ca / co, 3) if co else None,
                             "checksum_over_read_all": round(frac, 4) if frac else None,
                             "checksum_over_read_one": round(co / ro, 4) if ro else None,
                             "what": "oracle.read_probe: 64-bit word sums over the sample's own buffer, 4-KiB "
                                     "blocks split evenly over the leg's pinned workers, best of 3 runs of ~0.33 s"}
        # memory-bound when the checksum leg runs within 15 % of what the
        # same CPUs can merely read; otherwise the work bounds it
        out["bound"] = ("memory read path of these CPUs (the checksum leg runs at %.0f %% of a read-only pass "
                        "on the same CPUs)" % (100 * frac)) if frac and frac >= 0.85 else (
                        "checksum work (the same CPUs read the buffer %.2fx faster)" % (1 / frac) if frac else None)
    return out


def cpu_baseline(sample_fn, seconds: float, reps: int = 8, npk: int = 1 << 19, warm_max: float = 8.0):
    """The oracle (C restatement of checksum.cpp + a fastcsum-class nofold) on
    the host cores of this box, on a bounded sample of the same workload.
    All cores: `reps` repetitions of >= `seconds` each, the first dropped,
    the median of the rest is the value (min / max and every repetition beside
    it: a 16-core share of a 256-core host moves with its neighbours); one
    core: the same count of >= seconds / 2.  Worker thread t is pinned to the
    t-th CPU of the affinity mask (oracle/orc_pin.h)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import numpy as np
    import oracle  # test infrastructure: the CPU baseline leg only

    # 2^19 packets (~786 MB for 1500 B) by default, so the sample does not
    # sit in the host's last-level cache (EPYC 9575F: 256 MB L3) between
    # repetitions (npk / warm_max: smaller for the CPU test of this leg).
    host, gpu_out, kind = sample_fn(npk)
    cores = oracle.host_cores()
    threads = cores["threads"]
    # worker t on the t-th quietest CPU of the mask, one per physical core,
    # picked ONCE per leg and kept for all its repetitions (re-picking before
    # every repetition put the 1-core leg on cores of different speed:
    # bimodal values in round 4); oracle/orc_pin.h reads ORC_CPUS at every
    # thread start
    pin = os.environ.get("ORC_PIN", "1") != "0"
    picks = []

    def pick(n, policy="spread"):
        if pin:
            q = oracle.quiet_cpus(n, policy)
            os.environ["ORC_CPUS"] = ",".join(map(str, q["cpus"]))
            picks.append(q)
            return q["cpus"]
        return None

    reps_log = {"spread": [], "socket": [], "one": []}

    def logger(leg, cpus):
        # each repetition's CPUs and their clock right after it
        return lambda: reps_log[leg].append({"cpus": cpus, "cur_freq_khz": _cpu_freqs_khz(cpus) if cpus else None})

    cpus_all = pick(threads)
    quiet = picks[0] if picks else None
    # the sample's pages moved to the nodes of the workers that read them
    # (first touch by each pinned worker of its own share), per leg: the
    # sample was written by this thread, all on its node, and a worker on the
    # other socket read it remotely (round 6's first L3-spread lines: 17-22
    # GiB/s per socket-0 worker against 30-34 on socket 1)
    def retouch(n):
        if not pin:
            return None
        bufs = [host] + ([kind[3]] if kind[0] == "decap" else [])
        return all(isinstance(b, np.ndarray) and b.flags["C_CONTIGUOUS"] and b.flags["WRITEABLE"]
                   and oracle.numa_retouch(b, n) for b in bufs)

    numa_all = retouch(threads)
    one_scale = 1.0  # the 1-core leg runs on 1/one_scale of the sample
    extra = {}
    if kind[0] == "uniform":
        _, seg, cs, fl = kind
        exp = oracle.l4_uniform(host, seg, cs, fl, threads)
        run_all = lambda: oracle.l4_uniform(host, seg, cs, fl, threads)  # noqa: E731
        run_one = lambda: oracle.l4_uniform(host, seg, cs, fl, 1)  # noqa: E731
        nbytes = host.size
    elif kind[0] == "verify":
        d = kind[1]
        exp_v, exp_l4 = oracle.verify_desc(host, d, threads)
        run_all = lambda: oracle.verify_desc(host, d, threads)  # noqa: E731
        run_one = lambda: oracle.verify_desc(host, d, 1)  # noqa: E731
        nbytes = int(np.ascontiguousarray(d).view(oracle.PKT_DESC)["len"].astype(np.int64).sum())
        exp = np.concatenate([exp_v.astype(np.int64), exp_l4.astype(np.int64)])
        gpu_out = np.concatenate([gpu_out[0].astype(np.int64), gpu_out[1].astype(np.int64)])
    elif kind[0] == "gso":
        # do_tun_gso_split restatement per super-buffer, pthreads over
        # disjoint super-buffer ranges; the input prefix zeroing it does in
        # place is idempotent, so repetitions see the same bytes
        gk, out_bytes = kind[1], kind[2]
        cpu_out = np.zeros(out_bytes, np.uint8)
        st = oracle.gso_split_desc(host, gk, cpu_out, threads)
        exp = cpu_out.copy()
        sub = gk[: max(1, gk.size // 8)]
        one_scale = sub.size / gk.size
        run_all = lambda: oracle.gso_split_desc(host, gk, cpu_out, threads)  # noqa: E731
        run_one = lambda: oracle.gso_split_desc(host, sub, cpu_out, 1)  # noqa: E731
        nbytes = int(gk["in_len"].astype(np.int64).sum())
        npk = gk.size
        if np.any(st != 0):
            gpu_out = None  # a failed status is a parity failure
    elif kind[0] == "gro":
        d = kind[1]
        hdr_after, st = oracle.gro_finalize_desc(host, d, threads)
        exp = np.concatenate([hdr_after.astype(np.int64), st.astype(np.int64)])
        # timed: the C call only, in place on working copies made outside the
        # timed region (finalize is idempotent: re-running it on finalized
        # headers rewrites the same bytes)
        hw, dw = oracle.gro_working_copies(host, d)
        run_all = lambda: oracle.gro_finalize_desc_inplace(hw, dw, threads)  # noqa: E731
        run_one = lambda: oracle.gro_finalize_desc_inplace(hw, dw, 1)  # noqa: E731
        run_one()
        if not (np.array_equal(hw, hdr_after) and np.array_equal(dw["status"], st)):
            gpu_out = None  # the timed in-place runs must reproduce the checked answer
        nbytes = d.size  # flows
        if gpu_out is not None:
            gpu_out = np.concatenate([gpu_out[0].astype(np.int64), gpu_out[1].astype(np.int64)])
    elif kind[0] == "aead":
        # Peer::encrypt per segment: the oracle (scalar RFC 8439 restatement,
        # the bit-exact checker) and, as the stronger CPU comparator of
        # libsodium's class, the system OpenSSL's EVP_chacha20_poly1305
        _, key, rx, c0, seg = kind
        cpu_out = np.zeros(gpu_out.size + 64, np.uint8)
        oracle.wg_encrypt_batch_mt(key, rx, c0, host, seg, cpu_out, threads)
        exp = cpu_out[: gpu_out.size].copy()
        sub = host[: host.size // 8 // seg * seg]
        one_scale = sub.size / host.size
        run_all = lambda: oracle.wg_encrypt_batch_mt(key, rx, c0, host, seg, cpu_out, threads)  # noqa: E731
        run_one = lambda: oracle.wg_encrypt_batch_mt(key, rx, c0, sub, seg, cpu_out, 1)  # noqa: E731
        try:
            oss_all = _spread(_rep_rates(lambda: oracle.openssl_encrypt_batch(key, rx, c0, host, seg, cpu_out,
                                                                              threads), host.size, seconds, 4), 2.0**-30)
            oss_one = _spread(_rep_rates(lambda: oracle.openssl_encrypt_batch(key, rx, c0, sub, seg, cpu_out, 1),
                                         sub.size, seconds / 2, 4), 2.0**-30)
            extra = {"openssl_evp_chacha20_poly1305": {
                "value": oss_all["median"], "value_1core": oss_one["median"], "unit": "GiB/s",
                "spread": oss_all, "spread_1core": oss_one,
                "bit_exact_vs_oracle": bool(np.array_equal(cpu_out[: gpu_out.size], exp))}}
        except Exception as e:  # noqa: BLE001 - a comparator, never the checker
            extra = {"openssl_evp_chacha20_poly1305": f"unavailable: {e}"}
        nbytes = host.size
        npk = host.size // seg
    elif kind[0] == "encap":
        # do_tun_gso_split restatement (pthreads) then Peer::encrypt per
        # segment: exact messages for the parity check from the oracle per
        # super-buffer; timed: the split + OpenSSL's EVP ChaCha20-Poly1305
        # over the same segments as one batch (each super-buffer's shorter
        # last segment at full size: +0.3 % work)
        _, gk, out_bytes, key, rx, c0, seg, nseg, mcap, mbytes = kind
        seg_out = np.zeros(out_bytes, np.uint8)
        st = oracle.gso_split_desc(host, gk, seg_out, threads)
        exp = np.zeros(gk.size * mcap, np.uint8)
        ostride = out_bytes // gk.size
        for i in range(gk.size):
            ol = int(gk["in_len"][i]) - 40 + nseg * 40
            m = oracle.wg_encrypt_batch(key, rx, c0 + i * nseg, seg_out[i * ostride: i * ostride + ol], seg)
            exp[i * mcap: i * mcap + m.size] = m
            gpu_out[i * mcap + m.size: (i + 1) * mcap] = 0  # only the messages are compared
        segs = np.ascontiguousarray(seg_out.reshape(gk.size, ostride)[:, : nseg * seg]).reshape(-1)
        enc_out = np.zeros(gk.size * nseg * wga_stride(seg) + 64, np.uint8)
        sub = gk[: max(1, gk.size // 8)]
        ssub = segs[: sub.size * nseg * seg]
        one_scale = sub.size / gk.size

        def run_all():
            oracle.gso_split_desc(host, gk, seg_out, threads)
            oracle.openssl_encrypt_batch(key, rx, c0, segs, seg, enc_out, threads)

        def run_one():
            oracle.gso_split_desc(host, sub, seg_out, 1)
            oracle.openssl_encrypt_batch(key, rx, c0, ssub, seg, enc_out, 1)

        nbytes = int(gk["in_len"].astype(np.int64).sum())
        npk = gk.size
        if np.any(st != 0):
            gpu_out = None
    elif kind[0] == "decap":
        # Peer::decrypt + evaluate_packet per message: OpenSSL's EVP
        # ChaCha20-Poly1305 decrypt, then the verify-gate restatement over
        # the plaintexts (timed); parity against the oracle's decrypt + verify
        _, key, seg, msgs_host = kind
        n_m = (msgs_host.size + seg - 1) // seg
        pt, st = oracle.wg_decrypt_batch(key, msgs_host, seg)
        d = np.zeros(n_m, dtype=oracle.PKT_DESC)
        d["offset"] = np.arange(n_m, dtype=np.uint64) * (seg - 32)
        d["len"] = [min(seg, msgs_host.size - i * seg) - 32 for i in range(n_m)]
        ev, el4 = oracle.verify_desc(pt, d, threads)
        ev[st != 0], el4[st != 0] = 0, 0
        exp = np.concatenate([st.astype(np.int64), ev.astype(np.int64), el4.astype(np.int64)])
        gpu_out = np.concatenate([np.asarray(x).astype(np.int64) for x in gpu_out])
        pt_buf = np.zeros(n_m * (seg - 32) + 64, np.uint8)
        st_buf = np.zeros(n_m, np.int8)
        sub_m = msgs_host[: max(1, n_m // 8) * seg]
        one_scale = sub_m.size / msgs_host.size

        def run_all():
            oracle.openssl_decrypt_batch(key, msgs_host, seg, pt_buf, st_buf, threads)
            oracle.verify_desc(pt_buf, d, threads)

        def run_one():
            oracle.openssl_decrypt_batch(key, sub_m, seg, pt_buf, st_buf, 1)
            oracle.verify_desc(pt_buf, d[: sub_m.size // seg], 1)

        run_all()
        extra = {"openssl_decrypt_status_equal_oracle": bool(np.array_equal(st_buf, st))}
        nbytes = msgs_host.size
        npk = n_m
    elif kind[0] == "checksum":
        # checksum(buf, 0) per buffer (BASELINE config 1)
        d = kind[1]
        exp = oracle.checksum_desc(host, d, threads)
        run_all = lambda: oracle.checksum_desc(host, d, threads)  # noqa: E731
        run_one = lambda: oracle.checksum_desc(host, d, 1)  # noqa: E731
        nbytes = int(np.ascontiguousarray(d).view(oracle.PKT_DESC)["len"].astype(np.int64).sum())
        npk = d.size
    else:
        d = kind[1]
        exp = oracle.l4_desc(host, d, threads)
        run_all = lambda: oracle.l4_desc(host, d, threads)  # noqa: E731
        run_one = lambda: oracle.l4_desc(host, d, 1)  # noqa: E731
        nbytes = int(np.ascontiguousarray(d).view(oracle.PKT_DESC)["len"].astype(np.int64).sum())
    parity = gpu_out is not None and bool(np.array_equal(exp, gpu_out))
    scale, unit = (1e-6, "Mflows/s") if kind[0] == "gro" else (2.0**-30, "GiB/s")
    run_all()  # first touch / warm-up, untimed
    warm_log = {}

    def warm(name, fn, secs, secs_max=warm_max, tol=0.02):
        # untimed runs until the leg's pages have settled where its workers
        # run (round 5: repetitions still rose 30-60 % over the first
        # seconds on a 256-CPU host — page placement, not clocks: every
        # repetition's CPUs held the same scaling_cur_freq).  In 0.4-s
        # chunks: at least `secs`, then until two chunks in a row agree
        # within `tol`, at most `secs_max`.
        t0 = time.perf_counter()
        rates, prev = [], None
        while True:
            k, ts = 0, time.perf_counter()
            while time.perf_counter() - ts < 0.4:
                fn()
                k += 1
            rate = k / (time.perf_counter() - ts)
            rates.append(rate)
            el = time.perf_counter() - t0
            if el >= secs_max or (el >= secs and prev and abs(rate - prev) <= tol * prev):
                break
            prev = rate
        warm_log[name] = {"seconds": round(el, 2), "chunks": len(rates),
                          "last_rate_vs_first": round(rates[-1] / rates[0], 3)}

    probe_buf = host if isinstance(host, np.ndarray) and host.dtype == np.uint8 and host.size >= 1 << 20 else None

    def all_leg(policy, cpus, q, numa):
        # the all-core leg on one placement: CPUs dealt over the L3 domains of
        # the whole mask ("spread") or of one package ("socket"), the
        # sample's pages moved to those workers' nodes
        run_all()
        warm(f"all_{policy}", run_all, min(seconds, 1.5))
        thr0 = oracle.cgroup_throttling()
        oracle.pool_stats_reset()
        leg = _spread(_rep_rates(run_all, nbytes, seconds, reps, after=logger(policy, cpus)), scale)
        workers = oracle.pool_stats()
        thr1 = oracle.cgroup_throttling()
        read = _read_probe_rate(oracle, probe_buf, threads) if probe_buf is not None else None
        leg["repetitions"] = reps_log[policy]
        leg["warm_up"] = warm_log.get(f"all_{policy}")
        if thr0 and thr1:
            # CPU-quota throttling while the all-core repetitions ran (a share
            # of 16 CPUs leaves no room for a 17th busy thread)
            leg["cgroup_throttled"] = {k: thr1[k] - thr0[k] for k in thr0}
        return {"policy": policy, "spread": leg, "cpus": cpus, "quiet": q, "workers": workers, "read": read,
                "numa": numa}

    legs = [all_leg("spread", cpus_all, quiet, numa_all)]
    cpus_sock = pick(threads, "socket")
    if pin and set(cpus_sock or []) != set(cpus_all or []):
        legs.append(all_leg("socket", cpus_sock, picks[-1], retouch(threads)))
    best = max(legs, key=lambda L: L["spread"]["median"])
    all_s, cpus_all, quiet, workers, read_all = best["spread"], best["cpus"], best["quiet"], best["workers"], best["read"]
    numa_all = best["numa"]
    cpus_one = pick(1)
    numa_one = retouch(1)
    warm("one", run_one, min(seconds, 1.5))  # the 1-core leg's first touch on its CPU, untimed
    one_s = _spread(_rep_rates(run_one, nbytes * one_scale, seconds / 2, reps, after=logger("one", cpus_one)), scale)
    read_one = _read_probe_rate(oracle, probe_buf, 1) if probe_buf is not None else None
    placement = _placement_evidence(quiet, cpus_all, workers, nbytes, scale, unit, all_s, one_s, read_all, read_one,
                                    probe_buf)
    one_s["repetitions"] = reps_log["one"]
    one_s["warm_up"] = warm_log.get("one")
    placement["all_core_placements"] = {
        L["policy"]: {"value": L["spread"]["median"], "spread_pct": L["spread"]["spread_pct"], "cpus": L["cpus"],
                      "packages": (L["quiet"] or {}).get("packages"), "l3_domains": (L["quiet"] or {}).get("l3_domains"),
                      "read_probe_GiB_s": (L["read"] or {}).get("GiB_s")} for L in legs}
    placement["all_core_placement_used"] = best["policy"]
    try:
        cpu_model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:
        cpu_model = "unknown"
    what = {"verify": "decap verify gates restatement (orc_verify)", "gro": "GRO finalize restatement",
            "gso": "do_tun_gso_split restatement, output bytes compared",
            "checksum": "checksum(span, 0) restatement",
            "aead": "Peer::encrypt restatement over RFC 8439 (scalar C), message bytes compared",
            "encap": "do_tun_gso_split restatement + OpenSSL EVP ChaCha20-Poly1305 timed; messages compared with "
                     "the RFC 8439 restatement",
            "decap": "OpenSSL EVP ChaCha20-Poly1305 decrypt + verify-gate restatement timed; plaintext statuses, "
                     "verdicts and L4 results compared with the RFC 8439 restatement + orc_verify"}.get(
                kind[0], "calc_l4_checksum restatement")
    nofold = "AVX2 vector nofold (oracle/csum_oracle.c nofold_avx2)" if oracle.have_avx2() else "scalar nofold"
    return {
        "value": all_s["median"],
        "unit": unit,
        "cores": threads,
        "kind": "port",
        "value_1core": one_s["median"],
        "spread": all_s,
        "spread_1core": one_s,
        "cpu_model": cpu_model,
        "host_cores": dict(cores, pinned_cpus=quiet["cpus"] if quiet else None,
                           pinned_cpu_1core=cpus_one[0] if cpus_one else None,
                           pinned_cpus_busy_before=[q["busy"] for q in picks] if picks else None,
                           pinning="per leg, once before its repetitions: one worker per physical core, the "
                                   "L3 domains (CCDs) dealt round robin, quietest domain and quietest CPUs first "
                                   "(0.3-s /proc/stat sample), kept for every repetition of the leg; the all-core "
                                   "leg runs twice, over the domains of the whole mask and of one package, and "
                                   "reports the faster (all_core_placements)" if pin else "off"),
        "numa_first_touch": {"all": numa_all, "one": numa_one,
                             "what": "before each leg the sample's pages were dropped and copied back by that leg's "
                                     "pinned workers (oracle.numa_retouch), so each reads memory on its own node"},
        "all_core_placements": placement.get("all_core_placements"),
        "all_core_placement_used": placement.get("all_core_placement_used"),
        "l3_domains": placement.get("l3_domains"),
        "per_worker": placement.get("per_worker"),
        "read_probe": placement.get("read_probe"),
        "bound": placement.get("bound"),
        "sample": f"first {npk} units of the same batch, oracle/csum_oracle.c "
                  f"({what}; {nofold} for spans >= 256 B), {threads} pthreads "
                  f"(sched_getaffinity {cores['affinity']}, cgroup quota {cores['cgroup_quota_cpus']}); "
                  f"value = median of {reps - 1} repetitions of >= {seconds:.1f} s after a dropped first one "
                  f"(after untimed runs per leg: >= {min(seconds, 1.5):.1f} s, then until two 0.4-s chunks agree "
                  f"within 2 %, <= 8 s; spread.warm_up), "
                  f"1 core: the same of >= {seconds / 2:.1f} s; worker t pinned to the t-th least busy CPU of the "
                  f"affinity mask, one per physical core, picked once per leg (host_cores.pinning); "
                  f"bit-exact vs GPU: {parity}",
        "parity_with_gpu": parity,
        **extra,
    }


def load_traffic(workload: str):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary
    (profiles/pmc_<workload>.json, gfx950 FETCH_SIZE x2 correction applied
    there), or None if no such profile exists."""
    p = ROOT / "profiles" / f"pmc_{workload}.json"
    if not p.exists():
        return None
    try:
        return json.loads(p.read_text()).get("hbm_bytes_per_launch")
    except Exception:
        return None


# Peak VALU issue: one wave64 VALU instruction per 2 cycles per SIMD
# (MI355X_MICROARCH.md cycle constants, v_fma_f32 wave64 on SIMD-32), 1,024
# SIMDs at 2.4 GHz.
VALU_PEAK_WINST = 1024 * 2.4e9 / 2


def load_valu(workload: str):
    """VALU wave-instructions per launch of a VALU-bound workload's kernel
    from its committed rocprofv3 summary (profiles/valu_<workload>.json,
    SQ_INSTS_VALU), or None."""
    p = ROOT / "profiles" / f"valu_{workload}.json"
    if not p.exists():
        return None
    try:
        return json.loads(p.read_text())
    except Exception:
        return None


def valu_issue(valu, kernel: Optional[str], kern_ms: float, workload: str) -> dict:
    """The VALU issue roofline of a VALU-bound kernel (f4) from its committed
    instruction count, as roofline fields: {"valu_issue": ...}, or
    {"valu_issue_refused": why} when the profile counts another kernel than
    the timed one, or {} without a profile.  Every instruction is priced at
    one wave64 issue per 2 cycles of a SIMD (MI355X_MICROARCH.md), so
    multi-cycle operations make the true bound tighter than this fraction."""
    if not valu or not valu.get("valu_winst_per_launch"):
        return {}
    if kernel and valu.get("kernel") != kernel:
        return {"valu_issue_refused": f"profiles/valu_{workload}.json counts {valu.get('kernel')!r}, "
                                      f"the timed kernel is {kernel!r}"}
    ach = valu["valu_winst_per_launch"] / (kern_ms * 1e-3)
    return {"valu_issue": {
        "bound": "valu", "achieved": round(ach / 1e12, 4), "peak": round(VALU_PEAK_WINST / 1e12, 4),
        "unit": "T wave64-instructions/s", "frac": round(ach / VALU_PEAK_WINST, 4),
        "instructions_per_launch": valu["valu_winst_per_launch"],
        "source": f"profiles/valu_{workload}.json (rocprofv3 SQ_INSTS_VALU, {valu.get('kernel')})"}}


def post_checks(torch, wga, wl: Workload, world: int, dev, no_post: bool = False):
    """Outside the timed region: verify pass, result hash, RCCL gather."""
    from wireglider_amd import dist as wdist

    info = {}
    if wl.post is not None and not no_post:
        torch.cuda.synchronize()
        info.update(wl.post())
    if wl.out is None:
        return info
    torch.cuda.synchronize()
    h = wdist.allreduce_hash(wdist.result_hash(wl.out, wl.first_index), device=dev)
    info["result_hash"] = h
    t0 = time.perf_counter()
    full = wdist.gather_results(wl.out, wl.counts)
    torch.cuda.synchronize()
    info["gather_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    info["gathered_results"] = int(full.numel())
    # generate -> store -> verify (offload.cpp:202-204, evaluator.hpp:64,93)
    wga.store_l4csum(wl.buf, wl.desc, wl.out)
    ver = wga.calc_l4_checksum_desc(wl.buf, wl.desc)
    bad = torch.count_nonzero(ver.to(torch.int32)).to(torch.int64).reshape(1)
    import torch.distributed as dist

    if dist.is_initialized():
        dist.all_reduce(bad, op=dist.ReduceOp.SUM)
    info["verify_nonzero"] = int(bad.item())
    return info


def spawn_ranks(args) -> int:
    """--gpus N > 1 without a launcher: start N ranks under
    torch.distributed.run (rendezvous on 127.0.0.1) and return their exit
    status.  Runs before anything touches the GPU (torch.cuda.device_count()
    does not initialise it on this image), so the children own the devices."""
    import socket
    import subprocess

    import torch

    backend = os.environ.get("WG_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and ndev < args.gpus:
        print(f"bench.py: --gpus {args.gpus} but {ndev} GPU(s) visible (RCCL needs one GPU per rank; "
              "WG_DIST_BACKEND=gloo rehearses ranks sharing a GPU)", file=sys.stderr)
        return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def time_steps(torch, wl: Workload, args, world: int, dev) -> dict:
    """The timed region: barrier + synchronize, exactly K back-to-back
    launches with ONE HIP event pair on the launch stream at its two ends,
    synchronize + barrier; max over ranks.  Returns wall / kernel times."""
    import torch.distributed as dist

    from wireglider_amd import dist as wdist

    def barrier():
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize()

    settled = settle(torch, wl.launch, args.settle_seconds)
    for _ in range(args.warmup):
        wl.launch()
    barrier()
    # Events between the launches would each add a serialising marker:
    # ~6 us per step, 3 % of config 2 (repo:tools/gap_probe.py).
    stream = torch.cuda.current_stream()
    e_start, e_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    t0 = time.perf_counter()
    e_start.record(stream)
    for _ in range(args.steps):
        wl.launch()
    e_end.record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    kern_ms = e_start.elapsed_time(e_end) / args.steps
    # Cross-check for rocprofv3's per-dispatch durations (untimed): an event
    # pair around each launch, which also stops neighbouring launches from
    # overlapping at their boundaries.
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for x, y in evs:
        x.record(stream)
        wl.launch()
        y.record(stream)
    torch.cuda.synchronize()
    kern_ms_isolated = sum(x.elapsed_time(y) for x, y in evs) / args.steps
    wall = wdist.max_over_ranks(t1 - t0, dev)
    per_rank = wdist.all_gather_floats([kern_ms, t1 - t0, float(wl.payload_bytes)], dev)
    total_payload = sum(r[2] for r in per_rank)
    return {"settled": settled, "wall": wall, "kern_ms": kern_ms, "kern_ms_isolated": kern_ms_isolated,
            "kern_ms_per_rank": [round(r[0], 5) for r in per_rank],
            "wall_s_per_rank": [round(r[1], 6) for r in per_rank],
            "kern_ms_max": max(r[0] for r in per_rank), "total_payload": total_payload,
            "payload_per_rank": [r[2] for r in per_rank]}


def strong_scaling(torch, wga, args, rank: int, world: int, dev, name: str = "config5") -> dict:
    """A batch of fixed total size split across the ranks, timed like the
    main line: whole-job GiB/s = all ranks' packet bytes / max-over-ranks
    wall time.  config5: BASELINE config 5 (16,777,216 x 1500 B mixed v4/v6 x
    TCP/UDP, count = byte balance); config4strong: config 4's one bimodal
    64 B / 9000 B batch, split by bytes."""
    from wireglider_amd import dist as wdist

    wl = build_workload(wga, torch, name, rank, world, dev)
    torch.cuda.synchronize()
    t = time_steps(torch, wl, args, world, dev)
    h = wdist.allreduce_hash(wdist.result_hash(wl.out, wl.first_index), device=dev)
    out = {
        "workload": wl.cfg["workload"], "scaling": "strong", "packets_total": wl.cfg["packets_total"],
        "packets_per_rank": wl.counts,
        "bytes_per_rank": [int(b) for b in t["payload_per_rank"]],
        "value": round(t["total_payload"] * args.steps / t["wall"] * 2.0**-30, 3), "unit": "GiB/s",
        "ms_per_step": round(t["wall"] / args.steps * 1e3, 5),
        "kernel_ms_per_rank": t["kern_ms_per_rank"],
        "roofline_frac_rank0": round(wl.alg_bytes / (t["kern_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        # order-independent hash of all 16 M results: the same at every world
        # size when the sharded job is bit-exact
        "result_hash": h,
    }
    del wl
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    import torch
    import torch.distributed as dist

    import wireglider_amd as wga

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; WG_DIST_BACKEND=gloo (with ranks sharing a GPU)
    # only rehearses the multi-rank logic on a one-GPU box
    backend = os.environ.get("WG_DIST_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or args.force_dist:
        if world == 1:  # no launcher: a one-rank group on 127.0.0.1
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                import socket

                with socket.socket() as so:
                    so.bind(("127.0.0.1", 0))
                    os.environ["MASTER_PORT"] = str(so.getsockname()[1])
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        got = dist.get_world_size()
    else:
        got = 1
    grouped = dist.is_initialized()
    if grouped:
        # The group's first collectives initialise the communicator lazily,
        # and for the next ~25 ms the device runs this rank's kernels up to
        # 18 % slower (tools/dist_hiccup_probe.py, profiles/r05_dist_hiccup.json):
        # do them now, ahead of the workload's build and clock settling, so no
        # timed region sees it.
        for _ in range(3):
            dist.barrier()
            warm = torch.ones(1, dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(warm)
        torch.cuda.synchronize()
    if got != args.gpus:
        print(f"bench.py: process group has {got} rank(s) but --gpus {args.gpus}", file=sys.stderr)
        if grouped:
            dist.destroy_process_group()
        sys.exit(3)

    wl = build_workload(wga, torch, args.workload, rank, world, dev)
    torch.cuda.synchronize()
    t = time_steps(torch, wl, args, world, dev)
    wall, kern_ms = t["wall"], t["kern_ms"]

    ms_per_step = wall / args.steps * 1e3
    value = t["total_payload"] * args.steps / wall * wl.value_scale
    achieved = wl.alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = load_traffic(args.workload)
    pcie = None
    if wl.pcie:
        # host-memory workloads: the bound is PCIe, not HBM — the achieved
        # rate is the step's PCIe bytes over the wall time, against the raw
        # copy rates of this box (both directions at once: PCIe is full duplex)
        ceil = pcie_ceiling(torch, wl.pcie["h2d"], wl.pcie["d2h"])
        pb = wl.pcie["h2d"] + wl.pcie["d2h"]
        ach = pb / (wall / args.steps) / 1e9
        pcie = {"bound": "pcie", "achieved": round(ach, 2), "peak": ceil["both_GBps"], "unit": "GB/s",
                "frac": round(ach / ceil["both_GBps"], 4), "traffic": pb,
                "peak_source": "raw hipMemcpyAsync H2D + D2H of the step's bytes at once on two streams, pinned, "
                               "this box", "pcie_ceiling": ceil,
                "spec_peak_GBps": 128.0, "frac_of_spec": round(ach / 128.0, 4),
                "spec_source": "PCIe Gen5 x16: 64 GB/s per direction"}
    probe = measured_read_peak(torch, wga, wl.buf, run_bytes=wl.probe_run) if rank == 0 and not wl.pcie else None
    read_peak = probe["best"] if probe else None
    copy = None
    if rank == 0 and wl.copy_dst is not None:
        # the same-run read+write ceiling; the probe
        # overwrites the workload's output, so one more launch restores it
        # before the CPU baseline and post-checks read it
        copy = measured_copy_peak(torch, wga, wl.buf, wl.copy_dst)
        wl.launch()
        torch.cuda.synchronize()
    # The CPU baseline samples the batch as the timed launches saw it, so it
    # runs before post_checks (whose verify pass stores the checksums into the
    # packets).
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and wl.sample is not None:
        cpu = cpu_baseline(wl.sample, args.cpu_seconds)
    post = post_checks(torch, wga, wl, world, dev, args.no_post)
    meta = {"metric": wl.metric or "device-resident GiB/s, L4 checksum over packet batch; 1/2/4/8 MI355X",
            "pcie": pcie, "rw": wl.rw,
            "unit": wl.unit, "scaling": wl.scaling, "config": wl.cfg, "kernel": wl.kernel, "alg_bytes": wl.alg_bytes,
            "valu_kernel": wl.valu_kernel}
    del wl
    torch.cuda.empty_cache()
    strong = None if args.no_strong else strong_scaling(torch, wga, args, rank, world, dev)
    strong4 = None if args.no_strong else strong_scaling(torch, wga, args, rank, world, dev, "config4strong")
    line = {
        "metric": meta["metric"],
        "value": round(value, 3),
        "unit": meta["unit"],
        "n_gpus": got,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle_launches": t["settled"],
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": meta["scaling"],
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device-generated, seeded; BASELINE config shapes)",
        "config": meta["config"],
        "distributed": {"backend": dist.get_backend() if grouped else None, "world_size": got,
                        "kernel_ms_per_rank": t["kern_ms_per_rank"], "wall_s_per_rank": t["wall_s_per_rank"],
                        # the whole job against R x HBM peak (algorithmic
                        # bytes of every rank / the slowest rank's kernel time)
                        "frac_of_world_hbm_peak": round(meta["alg_bytes"] * got / (t["kern_ms_max"] * 1e-3)
                                                        / 1e9 / (HBM_PEAK_GBS * got), 4)},
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel": meta["kernel"],
            "alg_bytes_per_launch": meta["alg_bytes"],
            "traffic_source": f"profiles/pmc_{args.workload}.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, per launch)",
            # a REFERENCE POINT, not a ceiling: the same bytes read by
            # kernels with no checksum work, best variant of 3 passes; a
            # kernel that overlaps its loads better than the probe can exceed
            # it (round 5's config 2: 1.0085) — the ceiling is `peak`
            "read_probe_reference_GBps": round(read_peak, 1) if read_peak else None,
            "read_probe_variants": probe["variants"] if probe else None,
            "vs_read_probe_reference": round(achieved / read_peak, 4) if read_peak else None,
            "read_probe_note": "wg_probe_read over this workload's whole buffer in this run (contiguous 2/4/8-KiB "
                               "waves and, for <= 2-KiB packets, the L4 kernel's own issue structure); a reference "
                               "point that the kernel may exceed, not a ceiling" if read_peak else None,
            **({"measured_copy_peak": copy["best"], "copy_probe_variants": copy["variants"],
                "copy_probe_bytes_each_way": copy["bytes_each_way"],
                "frac_of_measured_copy_peak": round(achieved / copy["best"], 4),
                "copy_probe_note": "wg_probe_copy over this workload's own input and output buffers in this run, "
                                   "best variant of 3 passes; rate = bytes read + written per second, like "
                                   "`achieved`"} if copy else {}),
            "kernel_ms_avg": round(kern_ms, 5),
            "kernel_ms_avg_max_over_ranks": round(t["kern_ms_max"], 5),
            "kernel_ms_source": "HIP events at the two ends of the timed region on the launch stream / K "
                                "(back-to-back launches)",
            "kernel_ms_isolated": round(t["kern_ms_isolated"], 5),
            **({"read_bytes_per_launch": meta["rw"][0], "write_bytes_per_launch": meta["rw"][1],
                "read_achieved": round(meta["rw"][0] / (kern_ms * 1e-3) / 1e9, 2),
                "write_achieved": round(meta["rw"][1] / (kern_ms * 1e-3) / 1e9, 2),
                "read_write_note": "SURVEY §8(d): read-only and read+write rates stated separately; `achieved` is "
                                   "read + write"} if meta["rw"] else {}),
        },
        "post_checks": post,
    }
    line["roofline"].update(valu_issue(load_valu(args.workload), meta["valu_kernel"], kern_ms, args.workload))
    if meta["pcie"] is not None:
        # the device roofline does not apply to a host-memory pipeline
        line["roofline_device"] = line["roofline"]
        line["roofline"] = meta["pcie"]
    if strong is not None:
        line["strong_scaling"] = strong
        line["strong_scaling_config4"] = strong4
    if rank == 0:
        line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    if grouped:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
