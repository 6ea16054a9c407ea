#!/usr/bin/env python3
"""Does a process group slow the timed region, and where?  One rank (run it
under torch.distributed.run, or plain with --nogroup): config 2's launch
repeated in five timed regions exactly as bench.py times them (barrier +
synchronize, one event pair around K back-to-back launches), each region's
device ms per launch and the host time of each of its first launches.
Prints one JSON line."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch
    import torch.distributed as dist

    import bench
    import wireglider_amd as wga

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    backend = os.environ.get("WG_DIST_BACKEND", "nccl")
    group = "--nogroup" not in sys.argv
    if group:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    wl = bench.build_workload(wga, torch, "config2", 0, 1, dev)
    torch.cuda.synchronize()
    bench.settle(torch, wl.launch, 0.3)
    out = []
    for rep in range(5):
        for _ in range(5):
            wl.launch()
        if group:
            dist.barrier()
        torch.cuda.synchronize()
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        host = []
        e0.record(s)
        for _ in range(50):
            t = time.perf_counter()
            wl.launch()
            host.append((time.perf_counter() - t) * 1e6)
        e1.record(s)
        torch.cuda.synchronize()
        out.append({"rep": rep, "ms_per_launch": round(e0.elapsed_time(e1) / 50, 5),
                    "host_us_first5": [round(x, 1) for x in host[:5]], "host_us_max": round(max(host), 1),
                    "host_us_median": round(sorted(host)[25], 1)})
    print(json.dumps({"group": backend if group else None, "regions": out}), flush=True)
    if group:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
