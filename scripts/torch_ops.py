"""Which ATen ops still run inside a train step (names, shapes, counts, and the trainer source line that
issued them) -- torch.profiler, CPU side."""
import os
import sys
import types
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402
from torch.profiler import profile, ProfilerActivity  # noqa: E402

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
with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
    tr.train_step(x, m, y)
    torch.cuda.synchronize()
c = Counter()
for e in prof.events():
    if e.name in ("aten::add_", "aten::add", "aten::fill_", "aten::copy_", "aten::mul", "aten::zero_", "aten::zeros",
                  "aten::ones_like", "aten::mul_", "aten::sub", "aten::neg", "aten::div", "aten::clone",
                  "aten::contiguous", "aten::_to_copy", "aten::sum", "aten::mean", "aten::rsub", "aten::expand"):
        site = next((f for f in (e.stack or []) if "stcgan_amd" in f or "bench" in f), "?")
        c[(e.name, str(e.input_shapes)[:70], site.split("repo/")[-1][:90])] += 1
for (n, s, site), k in sorted(c.items(), key=lambda kv: -kv[1]):
    print(f"{k:4d} {n:16s} {s:70s} {site}")
