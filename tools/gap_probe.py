"""How much of a bench step is not kernel: K back-to-back launches of the
config 2 kernel timed by wall clock with and without a HIP event pair around
each launch (interleaved rounds)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
import wireglider_amd as wga  # noqa: E402

dev = torch.device("cuda:0")
wl = bench.build_workload(wga, torch, sys.argv[1] if len(sys.argv) > 1 else "config2", 0, 1, dev)
torch.cuda.synchronize()
bench.settle(torch, wl.launch, 0.3)
K = 100
stream = torch.cuda.current_stream()
res = {"events": [], "plain": [], "kernel_ms_events": []}
for _ in range(5):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        wl.launch()
        e1.record(stream)
    torch.cuda.synchronize()
    res["events"].append((time.perf_counter() - t0) / K * 1e3)
    res["kernel_ms_events"].append(sum(a.elapsed_time(b) for a, b in evs) / K)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        wl.launch()
    torch.cuda.synchronize()
    res["plain"].append((time.perf_counter() - t0) / K * 1e3)
print({k: [round(x, 5) for x in v] for k, v in res.items()})
