#!/usr/bin/env python3
"""Wall-clock probe of the host-memory steps (wg_encap_host / wg_decap_host,
bench.py workloads encap_host / decap_host): every call timed on its own
(each call drains its streams before returning), per host_chunk_mb value.
Run it in separate processes with and without HSA_ENABLE_SDMA=0 (all
copies by blit kernels), or WG_HOST_D2H=0..3 (large downloads by the
store kernel: bit 1 encap, bit 2 decap), to compare the copy paths.

usage: host_probe.py [encap_host|decap_host ...] [--chunks 64,128,256] [--calls 8]
"""
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    import bench
    import wireglider_amd as wga

    argv = sys.argv[1:]
    chunks, calls = [256], 8
    if "--chunks" in argv:
        i = argv.index("--chunks")
        chunks = [int(x) for x in argv[i + 1].split(",")]
        del argv[i:i + 2]
    if "--calls" in argv:
        i = argv.index("--calls")
        calls = int(argv[i + 1])
        del argv[i:i + 2]
    names = argv or ["encap_host", "decap_host"]
    dev = torch.device("cuda:0")
    saved = wga.tune_get("host_chunk_mb")
    for name in names:
        w = bench.build_workload(wga, torch, name, 0, 1, dev)
        for mb in chunks:
            wga.tune_set("host_chunk_mb", mb)
            w.launch()
            w.launch()
            ts = []
            for _ in range(calls):
                t0 = time.perf_counter()
                w.launch()
                ts.append((time.perf_counter() - t0) * 1e3)
            med = statistics.median(ts)
            print(json.dumps({"workload": name, "host_chunk_mb": mb, "sdma": os.environ.get("HSA_ENABLE_SDMA", "default"),
                              "host_d2h": wga.tune_get("host_d2h"), "ms_med": round(med, 3), "ms_all": [round(t, 2) for t in ts],
                              "GBps_pcie": round((w.pcie["h2d"] + w.pcie["d2h"]) / med / 1e6, 2),
                              "value": round(w.payload_bytes / (med * 1e-3) * w.value_scale, 3)}), flush=True)
        del w
        torch.cuda.empty_cache()
    wga.tune_set("host_chunk_mb", saved)
    ceil = bench.pcie_ceiling(torch, 1 << 31, 1 << 31)
    print(json.dumps({"pcie_ceiling_2GiB_each": ceil, "sdma": os.environ.get("HSA_ENABLE_SDMA", "default")}), flush=True)


if __name__ == "__main__":
    main()
