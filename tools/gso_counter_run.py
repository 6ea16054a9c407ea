"""Driver for tools/gso_counters.sh: a few GSO launches and copy-probe
launches over config 3 sized buffers."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
import wireglider_amd as wga  # noqa: E402

dev = torch.device("cuda:0")
wl = bench.build_workload(wga, torch, "config3", 0, 1, dev)
for _ in range(3):
    wl.launch()
src = torch.empty(17_179_869_184 // 2, dtype=torch.int16, device=dev)
dst = torch.empty_like(src)
for _ in range(3):
    wga.probe_copy(src, dst, 1)
torch.cuda.synchronize()
