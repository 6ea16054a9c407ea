#!/usr/bin/env python3
"""Interleaved A/B of the decap verify kernels (knob verify_small) over the
batch shapes a decap worker sees, one process, one device:
  1500B   1,048,576 x 1500 B mixed v4/v6 x TCP/UDP (bench.py --workload verify)
  64B     1,048,576 x 64 B mixed (TCP ACK-sized GRO batches)
  c4mix   config 4's 4,194,304 packets, 64 B / 9000 B 50/50 by a seeded draw
  alt     1,048,576 packets alternating 64 B / 1500 B in runs of 1-7 (small
          and long packets interleaved inside every 4-descriptor group)
  mixP    1,048,576 packets, P % of them 64 B at random among 1500-B ones
          (P = 3, 12, 25: where the per-call choice of verify_small = 7 flips)
Every packet carries a valid checksum.  Times are back-to-back launches
between one event pair (as bench.py), median of rounds; every variant's
verdicts and L4 results are compared with variant 0's.

usage: verify_ab.py [variant ...] [--rounds R] [--batches a,b,...]
  a variant is key=value[,key=value...] of wg_tune_set keys (default: the
  verify_small values 0, 7, 6, 8)
"""
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def build(wga, torch, dev, name):
    import numpy as np

    seed = 0x5EED00A1
    if name in ("1500B", "64B"):
        n, size = 1 << 20, (1500 if name == "1500B" else 64)
        buf = torch.empty(n * size, dtype=torch.uint8, device=dev)
        wga.synth_fill(buf, seed)
        desc = wga.synth_desc_stride(n, size, size, 1, seed, 0, device=dev)
        lens = np.full(n, size, np.int64)
    else:
        rng = np.random.default_rng(seed)
        if name == "c4mix":
            n = 1 << 22
            lens = np.where(rng.random(n) < 0.5, 64, 9000).astype(np.int64)
        elif name.startswith("mix"):  # mixP: P % of 64-B packets among 1500-B ones, placed at random
            n = 1 << 20
            lens = np.where(rng.random(n) < int(name[3:]) / 100, 64, 1500).astype(np.int64)
        else:
            n = 1 << 20
            runs = rng.integers(1, 8, n)
            cls = np.repeat(np.arange(runs.size) & 1, runs)[:n]
            lens = np.where(cls == 0, 64, 1500).astype(np.int64)
        offs = np.concatenate([[0], np.cumsum(lens[:-1])])
        fam = rng.integers(0, 4, n)
        raw = np.zeros((n, 2), dtype=np.int64)
        raw[:, 0] = offs
        cs = np.where(fam & 1, 40, 20)
        raw[:, 1] = lens | (cs << 32) | (fam.astype(np.int64) << 48)
        desc = torch.from_numpy(raw).to(dev)
        buf = torch.empty(int(offs[-1] + lens[-1]) + 16, dtype=torch.uint8, device=dev)
        wga.synth_fill(buf, seed)
    wga.synth_headers(buf, desc, seed, 0)
    wga.store_l4csum(buf, desc, wga.calc_l4_checksum_desc(buf, desc))
    torch.cuda.synchronize()
    alg = int(lens.sum()) + 19 * n  # bytes + 16-B descriptor + verdict + L4 result
    return buf, desc, n, alg


def main():
    import torch

    import bench
    import wireglider_amd as wga

    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    for opt in ("--rounds", "--batches"):
        if opt in sys.argv:
            args.remove(sys.argv[sys.argv.index(opt) + 1])
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 5
    specs = args or ["verify_small=0", "verify_small=7", "verify_small=6", "verify_small=8"]
    variants = [tuple((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.split(",")) for a in specs]
    keys = sorted({k for v in variants for k, _ in v})
    dev = torch.device("cuda:0")
    saved = {k: wga.tune_get(k) for k in keys}
    out = {}
    names = ("1500B", "64B", "c4mix", "alt", "mix3", "mix12", "mix25")
    if "--batches" in sys.argv:
        names = tuple(sys.argv[sys.argv.index("--batches") + 1].split(","))
    for name in names:
        buf, desc, n, alg = build(wga, torch, dev, name)
        verdict = torch.empty(n, dtype=torch.uint8, device=dev)
        l4 = torch.empty(n, dtype=torch.uint16, device=dev)
        times = {v: [] for v in variants}
        ref, exact, passing = None, {}, None

        def launch():
            wga.verify_desc(buf, desc, verdict=verdict, l4=l4)

        bench.settle(torch, launch, 0.2)
        for _ in range(rounds):
            for v in variants:
                for k in keys:
                    wga.tune_set(k, saved[k])
                for k, x in v:
                    wga.tune_set(k, x)
                for _ in range(3):
                    launch()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(20):
                    launch()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / 20)
                got = (verdict.clone(), l4.clone())
                if ref is None:
                    ref = got
                    passing = int(torch.count_nonzero((got[0] & 3) == 3).item())
                exact[v] = exact.get(v, True) and bool(torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]))
        out[name] = {"packets": n, "alg_bytes": alg, "packets_passing": passing,
                     "variants": {",".join(f"{k}={x}" for k, x in v): {
                         "ms_med": round(statistics.median(times[v]), 5), "ms_min": round(min(times[v]), 5),
                         "roofline_frac": round(alg / (statistics.median(times[v]) * 1e-3) / 8e12, 4),
                         "bit_exact_vs_first": exact[v]} for v in variants}}
        print(json.dumps({name: out[name]}), flush=True)
        del buf, desc, verdict, l4
        torch.cuda.empty_cache()
    for k in keys:
        wga.tune_set(k, saved[k])
    print(json.dumps({"verify_ab": out}), flush=True)


if __name__ == "__main__":
    main()
