"""First-layer conv (bs=32, 256x256x8 -> 128x128x64 + activation copies): the stem kernel (stc_conv_fwd_act) against
the im2col tile + stc_bn_apply, HIP events over 20 calls, and the HBM rate of the stem launch (compulsory bytes:
the input once, each output copy once)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import _lib as L, ops  # noqa: E402

BF = torch.bfloat16
dev = "cuda"


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


B, W = 32, 256
x = torch.randn((B, W, W, 8), device=dev).to(BF)
w = torch.randn((64, 8, 4, 4), device=dev) * 0.1
wp = ops.pack(L.PACK_CONV_FWD, w, 64, 8, BF)
Ho = W // 2
y1 = torch.empty((B, Ho, Ho, 64), device=dev, dtype=BF)
y2 = torch.empty((B, Ho, Ho, 128), device=dev, dtype=BF)
raw = torch.empty((B, Ho, Ho, 64), device=dev, dtype=BF)
for nout in (1, 2):
    y2v = L.nhwc_view(y2, 64) if nout == 2 else None
    t_stem = timed(lambda: ops.conv_act(L.CONV_S2, B, L.nhwc_view(x), 8, wp, 64, L.nhwc_view(y1), 0.2, BF, y2v, 0.0))
    t_conv = timed(lambda: ops.conv(L.CONV_S2, B, L.nhwc_view(x), 8, wp, 64, L.nhwc_view(raw), BF))
    t_two = timed(lambda: (ops.conv(L.CONV_S2, B, L.nhwc_view(x), 8, wp, 64, L.nhwc_view(raw), BF),
                           ops.bn_apply(B, L.nhwc_view(raw), 64, BF, None, L.nhwc_view(y1), 0.2, y2v, 0.0)))
    byt = B * W * W * 8 * 2 + nout * B * Ho * Ho * 64 * 2
    print(f"outputs {nout}: stem {t_stem:6.1f} us ({byt / t_stem / 1e6:.2f} TB/s)  im2col conv alone {t_conv:6.1f} us  "
          f"conv + bn_apply {t_two:6.1f} us", flush=True)

# the output layer's input gradient with the fused BN-backward sums (G: dq 8 ch -> 128 ch, BN on channels 64..127)
Cout, C = 128, 64
wt = torch.randn((8, Cout, 4, 4), device=dev) * 0.05
wd = ops.pack(L.PACK_CONVT_DGRAD, wt, Cout, 8, BF)
dq = torch.randn((B, W, W, 8), device=dev).to(BF)
bx = torch.randn((B, Ho, Ho, C), device=dev).to(BF)
out = torch.empty((B, Ho, Ho, Cout), device=dev, dtype=BF)
dx = torch.empty((B, Ho, Ho, C), device=dev, dtype=BF)
tabs = [torch.rand(C, device=dev) + 0.5 for _ in range(5)]
t_f = timed(lambda: ops.conv_bn_backward(L.CONV_S2, B, L.nhwc_view(dq), 8, wd, Cout, L.nhwc_view(out), BF,
                                         bn_x=L.nhwc_view(bx), C=C, bn_state=tuple(tabs[:4]), gamma=tabs[4], s_self=0.0,
                                         ch_off=64, dxv=L.nhwc_view(dx)))
byt = B * W * W * 8 * 2 + B * Ho * Ho * (Cout + C) * 2
print(f"BN-backward input gradient (stem + BN apply): {t_f:6.1f} us  (conv part compulsory {byt / 1e6:.0f} MB)", flush=True)

# the PatchGAN logits layer's input gradient with layer 4's BN-backward sums (dy 30x30x8 -> 31x31x512)
wt = torch.randn((8, 512, 4, 4), device=dev) * 0.05
ws1 = ops.pack(L.PACK_CONV_S1_DGRAD, wt, 512, 8, BF)
dy = torch.randn((B, 30, 30, 8), device=dev).to(BF)
bx = torch.randn((B, 31, 31, 512), device=dev).to(BF)
out = torch.empty((B, 31, 31, 512), device=dev, dtype=BF)
dx = torch.empty((B, 31, 31, 512), device=dev, dtype=BF)
tabs = [torch.rand(512, device=dev) + 0.5 for _ in range(5)]
t_l = timed(lambda: ops.conv_bn_backward(L.CONV_S1_DGRAD, B, L.nhwc_view(dy), 8, ws1, 512, L.nhwc_view(out), BF,
                                         bn_x=L.nhwc_view(bx), C=512, bn_state=tuple(tabs[:4]), gamma=tabs[4],
                                         s_self=0.2, dxv=L.nhwc_view(dx)))
t_a = timed(lambda: ops.bn_backward(B, L.nhwc_view(bx), 512, BF, L.nhwc_view(dx), g1=L.nhwc_view(out), s1=0.2,
                                    bn_state=tuple(tabs)))
print(f"logits-layer input gradient + BN backward: {t_l:6.1f} us (the BN-backward pair alone {t_a:6.1f} us)", flush=True)
