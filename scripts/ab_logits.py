"""The PatchGAN logits conv (31x31x512 -> 30x30x1 + bias, bs 32 bf16): the two-pass taps form (default) against the
tiled K-split kernel (force {4, 1}), HIP events over 20 calls, and their max difference."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import _lib as L, ops  # noqa: E402

BF = torch.bfloat16
dev = "cuda"
B = 32
x = torch.randn((B, 31, 31, 512), device=dev).to(BF)
w = ops.pack(L.PACK_CONV_FWD, torch.randn((1, 512, 4, 4), device=dev) * 0.02, 1, 512, BF)
b = torch.randn(1, device=dev)
outs, ts = [], []
for force in (None, (4, 1)):
    y = torch.empty((B, 1, 30, 30), device=dev)
    f = lambda: ops.conv(L.CONV_S1, B, L.nhwc_view(x), 512, w, 1, L.nchw_view(y), BF, bias=b, out_f32=True,  # noqa
                         force=force)
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        f()
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    outs.append(y.clone())
print(f"logits conv bs32: two-pass {ts[0]:.1f} us  tiled {ts[1]:.1f} us  max diff {float((outs[0] - outs[1]).abs().max()):.3e}"
      f" (scale {float(outs[1].abs().max()):.3e})", flush=True)
