"""Dump the bf16 weight gradients of the step's large wgrad problems (fixed seeds) to argv[1] (.npz),
with whichever library STC_LIB_PATH names: two runs with two libraries compared by
scripts/wgrad_dump.py --compare a.npz b.npz show whether a change to the split reduction is
bit-identical."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))

PROBS = [  # (B, s, dh, dw, gh, gw, R, Cg, Cg_out)
    (32, 2, 64, 64, 128, 128, 128, 64, 64),
    (32, 2, 32, 32, 64, 64, 256, 128, 128),
    (32, 1, 31, 31, 32, 32, 512, 256, 256),
    (32, 2, 8, 8, 16, 16, 512, 512, 512),
    (32, 2, 128, 128, 256, 256, 64, 8, 4),
]


def dump(path):
    import torch
    from stcgan_amd import _lib as L
    dev = torch.device("cuda", 0)
    lib = L.lib()
    out = {}
    for i, (B, s, dh, dw, gh, gw, R, Cg, Cg_out) in enumerate(PROBS):
        g = torch.Generator(device=dev).manual_seed(100 + i)
        d = (torch.randn((B, dh, dw, R), device=dev, generator=g) * 0.5).to(torch.bfloat16)
        x = (torch.randn((B, gh, gw, Cg), device=dev, generator=g) * 0.5).to(torch.bfloat16)
        dv, gv = L.nhwc_view(d), L.nhwc_view(x)
        ws_b = ctypes.c_int64()
        assert lib.stc_conv_wgrad_query(L.BF16, B, dh, dw, R, Cg, None, ctypes.byref(ws_b), None) == 0
        ws = torch.empty(max(int(ws_b.value), 16), dtype=torch.uint8, device=dev)
        dW = torch.empty((R, Cg_out, 4, 4), device=dev)
        rc = lib.stc_conv_wgrad_ex(L.BF16, B, s, dv, R, None, None, 0, 0.0, gv, Cg, Cg_out, None, None, 0, 0.0,
                                   L.ptr(dW), None, L.ptr(ws), int(ws_b.value), L.stream())
        assert rc == 0, lib.stc_last_error().decode()
        torch.cuda.synchronize()
        out[f"p{i}"] = dW.cpu().numpy()
    np.savez(path, **out)


def compare(a, b):
    A, Bz = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        same = np.array_equal(A[k].view(np.uint32), Bz[k].view(np.uint32))
        diff = float(np.abs(A[k] - Bz[k]).max())
        print(f"{k}: {'bit-identical' if same else 'DIFFERENT'} max|diff| {diff:.3e} max|v| {float(np.abs(A[k]).max()):.3e}")
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        dump(sys.argv[1])
