"""Host (Python) time per call site of the bf16 bs=32 train step: every public function of stcgan_amd.ops and the
engine's per-network entry points wrapped with inclusive perf_counter timers (thread-safe accumulation: the
backward runs on autograd's device thread, where cProfile does not look).  Prints ms per step and calls per step."""
import collections
import functools
import inspect
import os
import sys
import threading
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import engine, ops, optim, parallel  # noqa: E402
from stcgan_amd import _lib as L  # noqa: E402
from stcgan_amd.stcgan import STCGAN  # noqa: E402

acc = collections.defaultdict(float)
cnt = collections.Counter()
lock = threading.Lock()
depth = threading.local()


def wrap(mod, name, tag):
    f = getattr(mod, name)

    @functools.wraps(f)
    def g(*a, **k):
        d = getattr(depth, "d", 0)
        depth.d = d + 1
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            dt = time.perf_counter() - t
            depth.d = d
            with lock:
                acc[tag] += dt
                cnt[tag] += 1
                if d == 0:
                    acc["(top-level ops)"] += dt
    setattr(mod, name, g)


for name, f in list(vars(ops).items()):
    if inspect.isfunction(f) and not name.startswith("_") and f.__module__ == ops.__name__:
        wrap(ops, name, "ops." + name)
for name in ("gen_forward", "gen_backward", "disc_forward", "disc_backward"):
    wrap(engine, name, "engine." + name)
wrap(L, "nhwc_view", "L.nhwc_view")
for name in ("dest", "done", "flush"):
    wrap(engine.GradWriter, name, "GradWriter." + name)
wrap(engine._WgradLane, "run", "WgradLane.run")

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
acc.clear()
cnt.clear()
n = 10
t0 = time.perf_counter()
for _ in range(n):
    tr.train_step(x, m, y)
host = (time.perf_counter() - t0) / n
torch.cuda.synchronize()
print(f"host enqueue {host * 1e3:.2f} ms/step")
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"{v / n * 1e3:8.3f} ms {cnt[k] / n:7.1f} calls  {v / max(cnt[k], 1) * 1e6:7.1f} us/call  {k}")
