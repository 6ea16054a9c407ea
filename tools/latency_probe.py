#!/usr/bin/env python3
"""Small-batch latency of the batch entry points: synchronous call time
(launch + stream synchronise, median of 200) at growing batch sizes, for
  l4_uniform   calc_l4_checksum_batch over 1500-B v4/UDP segments
  l4_desc      calc_l4_checksum_desc over the same packets
  gso          gso_split of 64 KiB TCPV4 super-buffers (45 x 1460 B)
  aead         aead_encrypt_batch of 1500-B segments
Prints one JSON object.  The host side of the comparison is the per-core CPU
rate bench.py's cpu_baseline reports (profiles/r02_final_*_bench.json):
batch bytes / that rate is the 1-core time, and the crossover is where the
GPU call gets cheaper.
usage: latency_probe.py
"""
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def lat(torch, fn, reps=200):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 2)


def main():
    import numpy as np
    import torch

    import wireglider_amd as wga

    dev = torch.device("cuda:0")
    seg = 1500
    out = {}
    big = 1 << 15
    buf = torch.empty(big * seg, dtype=torch.uint8, device=dev)
    wga.synth_fill(buf, 9)
    desc_all = wga.synth_desc_stride(big, seg, seg, 1, 9, 0, device=dev)
    res = torch.empty(big, dtype=torch.uint16, device=dev)
    for n in (1, 8, 64, 512, 4096, 32768):
        view = buf[: n * seg]
        d = desc_all[:n]
        out.setdefault("l4_uniform", {})[n] = lat(torch, lambda: wga.calc_l4_checksum_batch(view, seg, False, False, 20,
                                                                                           out=res[:n]))
        out.setdefault("l4_desc", {})[n] = lat(torch, lambda: wga.calc_l4_checksum_desc(view, d, out=res[:n]))
        msgs = torch.empty(n * wga.aead_message_stride(seg), dtype=torch.uint8, device=dev)
        st = torch.empty(n, dtype=torch.int8, device=dev)
        out.setdefault("aead", {})[n] = lat(torch, lambda: wga.aead_encrypt_batch(view, seg, bytes(range(32)), 1, 0,
                                                                                  out=msgs, status=st))
    in_stride, out_stride, in_len = 65536, 73216, 65535
    nb = 512
    sb = torch.empty(nb * in_stride, dtype=torch.uint8, device=dev)
    wga.synth_fill(sb, 10)
    pd = np.zeros(nb, dtype=wga.PKT_DESC_DTYPE)
    pd["offset"] = np.arange(nb, dtype=np.uint64) * in_stride
    pd["len"], pd["csum_start"], pd["flags"] = in_len, 20, 2
    wga.synth_headers(sb, torch.from_numpy(pd.view(np.uint8).copy()).to(dev), 10, 0)
    gd = np.zeros(nb, dtype=wga.GSO_DESC_DTYPE)
    gd["in_offset"] = pd["offset"]
    gd["out_offset"] = np.arange(nb, dtype=np.uint64) * out_stride
    gd["in_len"], gd["out_cap"] = in_len, out_stride
    gd["vnet"]["flags"], gd["vnet"]["gso_type"], gd["vnet"]["gso_size"] = 1, 1, 1460
    gd["vnet"]["csum_start"], gd["vnet"]["csum_offset"] = 20, 16
    outb = torch.empty(nb * out_stride, dtype=torch.uint8, device=dev)
    gres = torch.empty(nb * wga.GSO_RESULT_BYTES, dtype=torch.uint8, device=dev)
    for n in (1, 8, 64, 512):
        dd = torch.from_numpy(gd[:n].view(np.uint8).copy()).to(dev)
        # the split rewrites each super-buffer's header prefix; re-running it
        # on its own output is still one full split per call (same geometry)
        out.setdefault("gso", {})[n] = lat(torch, lambda: wga.gso_split(sb, dd, outb, results=gres[: n * wga.GSO_RESULT_BYTES]),
                                           reps=100)
    print(json.dumps({"unit": "us per synchronous call (median)", "segment_bytes": seg, "gso_super_buffer_bytes": in_len,
                      "latency_us": out}), flush=True)


if __name__ == "__main__":
    main()
