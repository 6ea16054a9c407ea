#!/usr/bin/env python3
"""Host-memory path rate: the batch starts and ends in host
memory (tun / UDP socket buffers), so the end-to-end rate includes
hipMemcpyAsync H2D of the packets and D2H of the 2-byte results.

Measures, on BASELINE config 2 bytes (1,048,576 x 1500 B):
  pageable : wg_l4csum_uniform_host on a pageable numpy buffer (runtime staging)
  pinned   : the same entry point on a pinned (page-locked) host buffer
  pinned_pipelined : pinned buffer split into chunks, H2D of chunk k+1 overlapped
             with the kernel + D2H of chunk k on two streams
  h2d_only : hipMemcpyAsync of the pinned buffer alone (PCIe ceiling)
"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def main():
    import numpy as np
    import torch

    import wireglider_amd as wga

    n, seg = 1 << 20, 1500
    dev = torch.device("cuda:0")
    d = torch.empty(n * seg, dtype=torch.uint8, device=dev)
    wga.synth_fill(d, 0x5EED0002)
    desc = wga.synth_desc_stride(n, seg, seg, 0, 0x5EED0002, 0, device=dev)
    wga.synth_headers(d, desc, 0x5EED0002, 0)
    torch.cuda.synchronize()
    pageable = d.cpu().numpy()
    pinned = torch.empty(n * seg, dtype=torch.uint8, pin_memory=True)
    pinned.copy_(d.cpu())
    nbytes = n * seg
    out = {}

    def rate(fn, reps=5):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        return {"ms": round(dt * 1e3, 3), "GBps": round(nbytes / dt / 1e9, 2), "GiBps": round(nbytes / dt / 2**30, 2)}

    ref = wga.calc_l4_checksum_host(pageable, seg, False, False, 20)
    out["pageable"] = rate(lambda: wga.calc_l4_checksum_host(pageable, seg, False, False, 20))
    pv = pinned.numpy()
    got = wga.calc_l4_checksum_host(pv, seg, False, False, 20)
    assert np.array_equal(got, ref)
    out["pinned"] = rate(lambda: wga.calc_l4_checksum_host(pv, seg, False, False, 20))

    # two-stream chunked pipeline from pinned memory
    chunks = 16
    per = n // chunks
    dbuf = [torch.empty(per * seg, dtype=torch.uint8, device=dev) for _ in range(2)]
    dout = torch.empty(n, dtype=torch.uint16, device=dev)
    hout = torch.empty(n, dtype=torch.uint16, pin_memory=True)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def pipelined():
        for c in range(chunks):
            s = streams[c & 1]
            with torch.cuda.stream(s):
                b = dbuf[c & 1]
                b.copy_(pinned[c * per * seg:(c + 1) * per * seg], non_blocking=True)
                wga.calc_l4_checksum_batch(b, seg, False, False, 20, out=dout[c * per:(c + 1) * per], stream=s)
                hout[c * per:(c + 1) * per].copy_(dout[c * per:(c + 1) * per], non_blocking=True)
        torch.cuda.synchronize()

    pipelined()
    assert np.array_equal(hout.numpy(), ref)
    out["pinned_pipelined"] = rate(pipelined)
    out["h2d_only"] = rate(lambda: d.copy_(pinned, non_blocking=True))
    out["batch_bytes"] = nbytes
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
