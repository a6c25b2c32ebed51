"""Is the train step host-bound?  Host enqueue time of a step (no sync) vs its GPU time."""
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd.stcgan import STCGAN  # noqa: E402

a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                          D_loss_fn="standard", D_loss_type="normal", ngf=64, dtype="bf16", load_weights_g1=None,
                          load_weights_g2=None, load_weights_d1=None, load_weights_d2=None)
tr = STCGAN(a)
dev = torch.device("cuda", 0)
B = 32
x = torch.rand((B, 3, 256, 256), device=dev) * 2 - 1
m = (torch.rand((B, 1, 256, 256), device=dev) < 0.5).float() * 2 - 1
y = torch.rand((B, 3, 256, 256), device=dev) * 2 - 1
for _ in range(3):
    tr.train_step(x, m, y)
torch.cuda.synchronize()
# GPU-bound reference: many steps back to back
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0 = time.perf_counter()
e0.record()
for _ in range(10):
    tr.train_step(x, m, y)
t_host = (time.perf_counter() - t0) / 10
e1.record()
e1.synchronize()
t_wall = (time.perf_counter() - t0) / 10
print(f"host enqueue {t_host * 1e3:.2f} ms/step, wall {t_wall * 1e3:.2f} ms/step, gpu events {e0.elapsed_time(e1) / 10:.2f} ms/step")
# host time with the GPU idle at start (a sync before each step): does the GPU wait for the host?
ts = []
for _ in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train_step(x, m, y)
    ts.append(time.perf_counter() - t0)
print("host enqueue per step (after sync):", " ".join(f"{t * 1e3:.2f}" for t in ts), "ms")
# hidden synchronisation?  queue 100 ms of GPU sleep first: a step that syncs inside returns after it
torch.cuda.synchronize()
torch.cuda._sleep(int(2.4e9 * 0.1))
t0 = time.perf_counter()
tr.train_step(x, m, y)
t1 = time.perf_counter()
torch.cuda.synchronize()
print(f"after 100 ms of queued GPU sleep: step enqueue {1e3 * (t1 - t0):.2f} ms, drain {1e3 * (time.perf_counter() - t1):.2f} ms")
import cProfile, pstats  # noqa: E402,E401
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(3):
    tr.train_step(x, m, y)
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(18)
