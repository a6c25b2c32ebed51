"""Per-launch HIP-event timing of every conv-family launch of one ST-CGAN train step (bf16, bs=32)."""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import engine, ops  # noqa: E402
from stcgan_amd.stcgan import STCGAN  # noqa: E402

dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"
a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                          D_loss_fn="standard", D_loss_type="normal", ngf=64, dtype=dt, load_weights_g1=None,
                          load_weights_g2=None, load_weights_d1=None, load_weights_d2=None,
                          streams=False)  # one stream, no weight-gradient lane: each event pair brackets one kernel
engine.WGRAD_OVERLAP = False
tr = STCGAN(a)
dev = torch.device("cuda", 0)
B = 32
x = torch.rand((B, 3, 256, 256), device=dev) * 2 - 1
m = (torch.rand((B, 1, 256, 256), device=dev) < 0.5).float() * 2 - 1
y = torch.rand((B, 3, 256, 256), device=dev) * 2 - 1
for _ in range(2):
    tr.train_step(x, m, y)
torch.cuda.synchronize()
ops._timer = []
e0 = torch.cuda.Event(enable_timing=True)
e1 = torch.cuda.Event(enable_timing=True)
e0.record()
tr.train_step(x, m, y)
e1.record()
torch.cuda.synchronize()
tot = 0.0
for name, single, fl, a0, a1, desc in ops._timer:
    t = a0.elapsed_time(a1)
    tot += t
    print(f"{t * 1e3:8.1f} us {fl / 1e9:8.2f} GF {fl / (t * 1e-3) / 1e12:7.1f} TF {'  ' if single else '+R'} {name:42s} {desc}")
print(f"conv-family sum {tot:.2f} ms of step {e0.elapsed_time(e1):.2f} ms")
