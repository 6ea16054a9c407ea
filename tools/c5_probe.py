#!/usr/bin/env python3
"""Where does config 5 lose against config 2?  One process, one device:
config 5's 25 GB buffer and descriptors, timed as
  desc_split   the default descriptor kernel (split roles)
  desc_wpp     l4_small = 0 (wave per packet, descriptors prefetched)
  uniform      the same buffer as a uniform PacketBatch (stride 1500,
               csum_start 20: timing only, the results differ for v6 / TCP)
and the same three on the first 1,048,576 packets (config 2's size).
Median kernel ms over interleaved rounds (events on the launch stream);
GB/s of packet bytes.  usage: c5_probe.py [rounds]
"""
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

    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda:0")
    wl = bench.build_workload(wga, torch, "config5", 0, 1, dev)
    buf, desc, n = wl.buf, wl.desc, wl.n_units
    seg = bench.SEG
    small = 1 << 20
    outs = torch.empty(n, dtype=torch.uint16, device=dev)

    def v(name, nb, fn, knob=None):
        return (name, nb, fn, knob or {})

    variants = []
    for tag, m in (("full", n), ("1M", small)):
        b = buf[: m * seg]
        d = desc[:m]
        o = outs[:m]
        variants.append(v(f"desc_split_{tag}", m * seg, lambda b=b, d=d, o=o: wga.calc_l4_checksum_desc(b, d, out=o)))
        variants.append(v(f"desc_wpp_{tag}", m * seg, lambda b=b, d=d, o=o: wga.calc_l4_checksum_desc(b, d, out=o),
                          {"l4_small": 0}))
        variants.append(v(f"uniform_{tag}", m * seg,
                          lambda b=b, o=o: wga.calc_l4_checksum_batch(b, seg, False, False, 20, out=o)))
        variants.append(v(f"uniform_{tag}_4iter", m * seg,
                          lambda b=b, o=o: wga.calc_l4_checksum_batch(b, seg, False, False, 20, out=o),
                          {"l4_blocks": m // 64}))
    # grid-stride forms (C5_GRID=1): uniform with 16 iterations per wave,
    # wave-per-packet descriptors with 16
    import os
    b, d, o = buf, desc, outs
    if os.environ.get("C5_GRID") == "1":
        variants.append(v("uniform_full_blocks65536", n * seg,
                          lambda b=b, o=o: wga.calc_l4_checksum_batch(b, seg, False, False, 20, out=o),
                          {"l4_blocks": 65536}))
        variants.append(v("desc_wpp_full_blocks65536", n * seg,
                          lambda b=b, d=d, o=o: wga.calc_l4_checksum_desc(b, d, out=o),
                          {"l4_small": 0, "l4_blocks": 65536}))
    keys = sorted({k for *_, kn in variants for k in kn})
    dflt = {k: wga.tune_get(k) for k in keys}
    res = {name: [] for name, *_ in variants}
    st = torch.cuda.current_stream()
    for r in range(rounds):
        for name, nb, fn, knob in variants:
            for k in keys:
                wga.tune_set(k, knob.get(k, dflt[k]))
            reps = 10 if "full" in name else 100
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(reps):
                fn()
            e1.record(st)
            e1.synchronize()
            res[name].append(e0.elapsed_time(e1) / reps)
        print(f"round {r} done", flush=True)
    for k in keys:
        wga.tune_set(k, dflt[k])
    out = {}
    for name, nb, *_ in variants:
        ms = statistics.median(res[name])
        out[name] = {"ms": round(ms, 5), "GBs": round(nb / ms / 1e6, 1), "all": [round(x, 5) for x in res[name]]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
