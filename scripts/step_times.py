"""Per-step wall times of the bench workload (bench.make_trainer, bs=32 bf16) from the first step on: how many
steps the trainer needs before it reaches its steady state (lazy tables, allocator growth, lane carry-over)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
torch.manual_seed(1234)
tr = bench.make_trainer(64, "bf16", 0)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(1234)
x = torch.rand((32, 3, 256, 256), generator=g, device=dev) * 2 - 1
m = (torch.rand((32, 1, 256, 256), generator=g, device=dev) < 0.5).float() * 2 - 1
y = torch.rand((32, 3, 256, 256), generator=g, device=dev) * 2 - 1
ts = []
for i in range(n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train_step(x, m, y)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
print(" ".join(f"{t:.2f}" for t in ts))
for w in (3, 5, 10):
    for k in (10, 20):
        if w + k <= n:
            print(f"warmup {w} steps {k}: synced per-step mean {sum(ts[w:w + k]) / k:.3f} ms")
t0 = time.perf_counter()
for _ in range(10):
    tr.train_step(x, m, y)
torch.cuda.synchronize()
print(f"then 10 back-to-back steps: {(time.perf_counter() - t0) * 100:.3f} ms/step")
