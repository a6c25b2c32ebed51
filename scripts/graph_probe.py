"""How fast is the train step with no host in the loop?  Capture one bf16 bs=32 step (side streams
included) into a HIP graph and time replays against eager steps.  Timing probe only (the optimizer steps are
timed eagerly, outside the graph)."""
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
                          load_weights_g2=None, load_weights_d1=None, load_weights_d2=None,
                          streams=os.environ.get("LANES", "1") == "1")
tr = STCGAN(a)
dev = torch.device("cuda", 0)
B = 32
x = torch.rand((B, 3, 256, 256), device=dev) * 2 - 1
m = (torch.rand((B, 1, 256, 256), device=dev) < 0.5).float() * 2 - 1
y = torch.rand((B, 3, 256, 256), device=dev) * 2 - 1


def timed(fn, n):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        tr.train_step(x, m, y)
torch.cuda.current_stream().wait_stream(s)
print(f"eager: {timed(lambda: tr.train_step(x, m, y), 10):.3f} ms/step", flush=True)
# the optimizer steps upload a pointer table from pinned memory (not capturable): capture the
# forwards/backwards only and time the two Adam steps eagerly
opt_steps = (tr.optim_D.step, tr.optim_G.step)
print(f"eager optimizer steps: {timed(lambda: (opt_steps[0](), opt_steps[1]()), 10):.3f} ms/step", flush=True)
tr.optim_D.step = tr.optim_G.step = lambda: None
print(f"eager without optimizer: {timed(lambda: tr.train_step(x, m, y), 10):.3f} ms/step", flush=True)
g = torch.cuda.CUDAGraph()
t0 = time.perf_counter()
with torch.cuda.graph(g):
    tr.train_step(x, m, y)
torch.cuda.synchronize()
print(f"captured in {time.perf_counter() - t0:.2f} s", flush=True)
print(f"graph replay: {timed(g.replay, 20):.3f} ms/step", flush=True)
print(f"eager without optimizer again: {timed(lambda: tr.train_step(x, m, y), 10):.3f} ms/step", flush=True)
