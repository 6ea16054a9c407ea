#!/usr/bin/env python3
"""Interleaved A/B of GSO split kernel variants on BASELINE config 3, one
process.  usage: ab_gso.py [key=value[,key=value...] ...]  (wg_tune_set keys,
e.g. gso_waves=8,gso_spw=2; a bare number means gso_ablate)."""
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    import bench
    import wireglider_amd as wga

    def parse(a):
        if "=" not in a:
            return (("gso_ablate", int(a)),)
        return tuple((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.split(","))

    vals = [parse(a) for a in sys.argv[1:]] or [parse("0"), parse("32")]
    defaults = {"gso_ablate": 0, "gso_waves": 4, "gso_spw": 1, "gso_split": 1}
    dev = torch.device("cuda:0")
    wl = bench.build_workload(wga, torch, "config3", 0, 1, dev)
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
    out = {",".join(f"{k}={x}" for k, x in v): {"ms_med": round(statistics.median(t), 4),
                    "GBps": round(wl.alg_bytes / (statistics.median(t) * 1e-3) / 1e9, 1)} for v, t in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
