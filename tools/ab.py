#!/usr/bin/env python3
"""Interleaved A/B of launch-geometry variants (wg_tune_set keys) on one
bench.py workload, one process, one device.

usage: ab.py <workload> [key=value[,key=value...] ...]
  e.g. ab.py config3 gso_groups=1 gso_groups=6 gso_groups=12,gso_waves=8
       ab.py config5 l4_small=0 l4_small=5
Every variant starts from the library's defaults; rounds interleave the
variants so clock / thermal drift hits them alike.  Prints one JSON object:
variant -> median kernel ms and algorithmic GB/s.
"""
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

KEYS = ("l4_blocks", "l4_nt", "l4_small", "l4_small_uniform", "verify_small", "verify_auto_t", "verify_k2min",
        "gso_blocks", "gso_waves", "gso_split", "gso_spw", "encap_spw", "gso_groups", "gso_ablate", "l4_unroll",
        "host_chunk_mb", "l4_coop", "l4_coop_waves", "aead_k", "aead_stage", "encap_parts", "encap_synth", "host_d2h", "lane_coop")


def main():
    import torch

    import bench
    import wireglider_amd as wga

    workload = sys.argv[1]
    vals = [tuple((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.split(",")) for a in sys.argv[2:]] or [()]
    defaults = {k: wga.tune_get(k) for k in KEYS}
    dev = torch.device("cuda:0")
    wl = bench.build_workload(wga, torch, workload, 0, 1, dev)
    torch.cuda.synchronize()
    bench.settle(torch, wl.launch, 0.3)
    res = {v: [] for v in vals}
    for _ in range(4):
        for v in vals:
            for key, val in defaults.items():
                wga.tune_set(key, val)
            for key, val in v:
                wga.tune_set(key, val)
            wl.launch()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for e0, e1 in ev:
                e0.record()
                wl.launch()
                e1.record()
            torch.cuda.synchronize()
            res[v] += [e0.elapsed_time(e1) for e0, e1 in ev]
    for key, val in defaults.items():
        wga.tune_set(key, val)
    out = {",".join(f"{k}={x}" for k, x in v) or "default": {
        "ms_med": round(statistics.median(t), 4),
        "GBps": round(wl.alg_bytes / (statistics.median(t) * 1e-3) / 1e9, 1)} for v, t in res.items()}
    print(json.dumps({"workload": workload, "alg_bytes": wl.alg_bytes, "variants": out}), flush=True)


if __name__ == "__main__":
    main()
