"""A/B in one process: Adam + lazy multi-tensor repack vs the fused stc_adam_pack_step, on the
generators' real parameter set (ngf=64, bf16 operands)."""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import ops  # noqa: E402
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
for _ in range(2):
    tr.train_step(x, m, y)
torch.cuda.synchronize()
opt = tr.optim_G


def run(fused, reps=10):
    opt.fuse_pack = fused
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for it in range(reps + 2):
        if it == 2:
            e0.record()
        opt.step()
        if not fused:
            for net in (tr.G1, tr.G2):
                ops.refresh_packs(net._pack_cache)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for _ in range(2):
    print(f"unfused (adam + refresh_packs): {run(False):8.1f} us   fused adam_pack: {run(True):8.1f} us")
