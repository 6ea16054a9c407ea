#!/usr/bin/env python3
"""Is a workload's kernel time a property of its buffer's placement?

usage: placement_probe.py <workload> [allocations]
       (env PROBE_K launches per timing, PROBE_SETTLE warm-up seconds: small
       values under rocprofv3 --pmc, which serialises every dispatch)
Builds the bench.py workload `allocations` times in one process (each new
buffer allocated while the previous one is still held, so each lands at a
new address, then the previous is released), and times 20 launches of each
with HIP events, interleaving rounds over the live ones (at most 2).  Prints
one JSON object: per allocation the buffer address and the median ms.
"""
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


K = int(__import__("os").environ.get("PROBE_K", "20"))          # launches per timing
SETTLE = float(__import__("os").environ.get("PROBE_SETTLE", "0.3"))  # seconds of warm-up launches


def time_wl(torch, wl, k=None):
    k = k or K
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
    for e0, e1 in ev:
        e0.record()
        wl.launch()
        e1.record()
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in ev]


def probe_whole(torch, wga, buf, run_bytes, k=5):
    """The kernel-shaped read probe over the WHOLE buffer (4 GiB slices):
    GB/s of a no-work read of the same physical pages."""
    acc = torch.zeros(1, dtype=torch.int64, device=buf.device)
    step = (4 << 30) // (16 * run_bytes) * 16 * run_bytes if run_bytes else 4 << 30  # slices stay 16-B aligned
    views = [buf[o: min(o + step, buf.numel()) // 16 * 16] for o in range(0, buf.numel(), step)]
    views = [v for v in views if v.numel() >= 4096]

    def once():
        for v in views:
            wga.probe_read(v, acc, 1 if run_bytes else 4, run_bytes=run_bytes)

    once()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        once()
    e1.record()
    torch.cuda.synchronize()
    nb = sum(v.numel() // run_bytes * run_bytes if run_bytes else v.numel() for v in views)
    return round(nb * k / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)


def main():
    import torch

    import bench
    import wireglider_amd as wga

    name = sys.argv[1]
    nalloc = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device("cuda:0")
    out = []
    prev = None
    for a in range(nalloc):
        wl = bench.build_workload(wga, torch, name, 0, 1, dev)
        torch.cuda.synchronize()
        if SETTLE > 0:
            bench.settle(torch, wl.launch, SETTLE)
        cur = time_wl(torch, wl)
        rec = {"alloc": a, "ptr": hex(wl.buf.data_ptr()), "ms_med": round(statistics.median(cur), 4),
               "GBps": round(wl.alg_bytes / (statistics.median(cur) * 1e-3) / 1e9, 1)}
        if wl.probe_run:
            rec["probe_whole_GBps"] = probe_whole(torch, wga, wl.buf, wl.probe_run)
        if prev is not None:  # the previous allocation again, right after: drift vs placement
            rec["prev_again_ms_med"] = round(statistics.median(time_wl(torch, prev)), 4)
            rec["this_again_ms_med"] = round(statistics.median(time_wl(torch, wl)), 4)
        out.append(rec)
        print(json.dumps(rec), flush=True)
        prev = None
        torch.cuda.empty_cache()
        prev = wl
    print(json.dumps({"workload": name, "allocations": out}), flush=True)


if __name__ == "__main__":
    main()
