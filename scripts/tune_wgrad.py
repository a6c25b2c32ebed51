"""Plan sweep of the bf16 weight-gradient kernel (csrc/wgrad_bf16.hip) over every wgrad problem of
one ST-CGAN train step (bs=32, 256x256).  Records the problems by running one step with a hook on
ops.wgrad, then times each forced (tile config, pixel splits) with HIP events over a captured HIP
graph.  Prints one line per problem: the auto plan's time and the best forced plan.
Output: JSON to argv[1]."""
import ctypes
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))

import torch  # noqa: E402

from stcgan_amd import _lib as L  # noqa: E402
from stcgan_amd import ops  # noqa: E402
from stcgan_amd.stcgan import STCGAN  # noqa: E402

BF = torch.bfloat16
CFGS = range(9)
SPLITS = tuple(int(v) for v in os.environ.get("WG_SPLITS", "0,1,2,4,8,16,32,64").split(","))
MIN_P = int(os.environ.get("WG_MIN_P", "0"))
WG_CFGS = os.environ.get("WG_CFGS")
if WG_CFGS:
    CFGS = tuple(int(v) for v in WG_CFGS.split(","))


def record():
    probs = {}
    orig = ops.wgrad

    def wgrad(B, stride, Dv, R, Gv, Cg, Cg_out, dt, dpro=None, dslope=None, gpro=None, gslope=None, device=None,
              **kw):
        if (dt == BF and dpro is None and gpro is None and dslope is None and gslope is None
                and not (kw.get("rows") and kw["rows"] < R)):
            k = (B, stride, Dv.H, Dv.W, Gv.H, Gv.W, R, Cg, Cg_out)
            probs[k] = probs.get(k, 0) + 1
        return orig(B, stride, Dv, R, Gv, Cg, Cg_out, dt, dpro, dslope, gpro, gslope, device, **kw)

    ops.wgrad = wgrad
    a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                              D_loss_fn="standard", D_loss_type="normal", ngf=64, dtype="bf16",
                              load_weights_g1=None, load_weights_g2=None, load_weights_d1=None,
                              load_weights_d2=None)
    tr = STCGAN(a)
    dev = torch.device("cuda", 0)
    B = 32
    x = torch.rand((B, 3, 256, 256), device=dev) * 2 - 1
    m = (torch.rand((B, 1, 256, 256), device=dev) < 0.5).float() * 2 - 1
    y = torch.rand((B, 3, 256, 256), device=dev) * 2 - 1
    tr.train_step(x, m, y)
    torch.cuda.synchronize()
    ops.wgrad = orig
    return probs


def bench(prob, force, reps=10):
    """Time (us) of one stc_conv_wgrad call (kernel + split reduction) under a forced plan."""
    B, s, dh, dw, gh, gw, R, Cg, Cg_out = prob
    dev = torch.device("cuda", 0)
    d = (torch.randn((B, dh, dw, R), device=dev) * 0.5).to(BF)
    g = (torch.randn((B, gh, gw, Cg), device=dev) * 0.5).to(BF)
    dv, gv = L.nhwc_view(d), L.nhwc_view(g)
    lib = L.lib()
    fp = None if force is None else (ctypes.c_int32 * 2)(*force)
    ws_b = ctypes.c_int64()
    if lib.stc_conv_wgrad_query(L.BF16, B, dh, dw, R, Cg, fp, ctypes.byref(ws_b), None) != 0:
        return None
    nbytes = ws_b.value
    ws = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=dev)
    dW = torch.empty((R, Cg_out, 4, 4), device=dev)

    def call():
        rc = lib.stc_conv_wgrad_ex(L.BF16, B, s, dv, R, None, None, 0, 0.0, gv, Cg, Cg_out, None, None, 0, 0.0,
                                   L.ptr(dW), fp, L.ptr(ws), int(nbytes), L.stream())
        if rc != 0:
            raise RuntimeError(lib.stc_last_error().decode())

    try:
        call()
        torch.cuda.synchronize()
    except RuntimeError:
        return None
    gr = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        with torch.cuda.graph(gr, stream=st):
            for _ in range(reps):
                call()
    torch.cuda.synchronize()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gr.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    probs = record()
    out = []
    tot_auto = tot_best = 0.0
    for prob, count in sorted(probs.items(), key=lambda kv: -kv[0][0] * kv[0][2] * kv[0][3] * kv[0][6] * kv[0][7]):
        B, s, dh, dw, gh, gw, R, Cg, Cg_out = prob
        if B * dh * dw < MIN_P:
            continue
        flops = 2.0 * B * dh * dw * R * 16 * Cg
        t_auto = bench(prob, (-1, 0))
        res = {}
        for cfg in CFGS:
            for ns in SPLITS:
                t = bench(prob, (cfg, ns), reps=5)
                if t is not None:
                    res[(cfg, ns)] = t
        best = min(res, key=res.get)
        tot_auto += t_auto * count
        tot_best += res[best] * count
        print(f"wgrad s{s} P={B * dh * dw:7d} R={R:4d} Cg={Cg:4d} n={count}  auto {t_auto:8.1f}us "
              f"{flops / t_auto / 1e6:7.1f}TF | best cfg{best[0]},ns{best[1]} {res[best]:8.1f}us "
              f"{flops / res[best] / 1e6:7.1f}TF", flush=True)
        out.append({"prob": prob, "count": count, "auto": t_auto, "best": [best[0], best[1], res[best]],
                    "all": {f"{k[0]},{k[1]}": v for k, v in res.items()}})
    print(f"sum over one step: auto {tot_auto / 1e3:.2f} ms, best {tot_best / 1e3:.2f} ms")
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
