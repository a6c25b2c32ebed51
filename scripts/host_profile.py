"""cProfile of the host side of 5 bf16 bs=32 train steps (after warm-up): where the enqueue time goes."""
import cProfile
import os
import pstats
import sys
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
x = torch.rand((32, 3, 256, 256), device=dev) * 2 - 1
m = (torch.rand((32, 1, 256, 256), device=dev) < 0.5).float() * 2 - 1
y = torch.rand((32, 3, 256, 256), device=dev) * 2 - 1
for _ in range(3):
    tr.train_step(x, m, y)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    tr.train_step(x, m, y)
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)
