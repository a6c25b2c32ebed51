"""Step time from a cold start: the bench workload's train steps timed in consecutive windows of 10 (first process
on a box: does the GPU need longer than the bench's warm-up to reach its steady step time?)."""
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
torch.manual_seed(1234)
tr = STCGAN(a)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(1234)
x = torch.rand((32, 3, 256, 256), generator=g, device=dev) * 2 - 1
m = (torch.rand((32, 1, 256, 256), generator=g, device=dev) < 0.5).float() * 2 - 1
y = torch.rand((32, 3, 256, 256), generator=g, device=dev) * 2 - 1
torch.cuda.synchronize()
t_start = time.perf_counter()
for w in range(int(sys.argv[1]) if len(sys.argv) > 1 else 30):
    t0 = time.perf_counter()
    for _ in range(10):
        tr.train_step(x, m, y)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    print(f"window {w:3d} (t={t0 - t_start:6.2f} s): {(t1 - t0) / 10 * 1e3:7.3f} ms/step", flush=True)
