"""Tile-plan sweep of the bf16 LDS-DMA implicit GEMM over every conv problem of one ST-CGAN
train step (bs=32, 256x256).  Records the problems by running one step with a hook on ops.conv /
ops.conv_stats, then times each (tile config, ksplit) with HIP events on the current stream.
Prints one line per problem: the auto plan's time and the best forced plan.  Output: JSON to argv[1]."""
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
NCFG = 36


def record():
    probs = {}
    orig_conv, orig_stats = ops.conv, ops.conv_stats

    def key(kind, B, xv, cin, cout, yv):
        gh, gw = (xv.H, xv.W) if kind == L.CONVT_S2 else (yv.H, yv.W)
        return (kind, B, gh, gw, xv.H, xv.W, yv.H, yv.W, cin, cout)

    def conv(kind, B, xv, cin, w, cout, yv, dt, **kw):
        if kw.get("pro") is None and not kw.get("out_f32") and yv.cs == 1:
            probs.setdefault(key(kind, B, xv, cin, cout, yv), [0, False])[0] += 1
        return orig_conv(kind, B, xv, cin, w, cout, yv, dt, **kw)

    def conv_stats(kind, B, xv, cin, w, cout, yv, dt, **kw):
        e = probs.setdefault(key(kind, B, xv, cin, cout, yv), [0, True])
        e[0] += 1
        e[1] = True
        return orig_stats(kind, B, xv, cin, w, cout, yv, dt, **kw)

    ops.conv, ops.conv_stats = conv, conv_stats
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
    ops.conv, ops.conv_stats = orig_conv, orig_stats
    return probs


def bench(prob, force, reps=10):
    """Kernel time (us) of one conv_stats call, from a captured HIP graph of `reps` calls."""
    import ctypes
    kind, B, gh, gw, xh, xw, yh, yw, cin, cout = prob
    dev = torch.device("cuda", 0)
    x = (torch.randn((B, xh, xw, cin), device=dev) * 0.5).to(BF)
    y = torch.empty((B, yh, yw, cout), device=dev, dtype=BF)
    taps = 4 if kind == L.CONVT_S2 else 16
    nph = 4 if kind == L.CONVT_S2 else 1
    w = (torch.randn((nph, cout, taps, cin), device=dev) * 0.05).to(BF)
    xv, yv = L.nhwc_view(x), L.nhwc_view(y)
    try:
        nbytes, nch, plan = ops.conv_query(kind, B, gh, gw, cin, cout, BF, force=force)
    except RuntimeError:
        return None
    ws = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=dev)
    part = torch.empty((nch, cout, 4), device=dev)
    fp = (ctypes.c_int32 * 2)(*force) if force is not None else None
    lib = L.lib()

    def call():
        rc = lib.stc_conv_fwd_ex(L.BF16, kind, B, xv, cin, L.ptr(w), cout, yv, None, 0, 0, L.ptr(part), nch, fp,
                                 L.ptr(ws), int(nbytes), L.stream())
        if rc != 0:
            raise RuntimeError(lib.stc_last_error().decode())

    try:
        call()
        torch.cuda.synchronize()
    except RuntimeError:
        return None
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                call()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    probs = record()
    out = []
    names = {0: "conv_s2", 1: "conv_s1", 2: "convT", 3: "s1_dgrad"}
    tot_auto = tot_best = 0.0
    for prob, (count, _) in sorted(probs.items(), key=lambda kv: -kv[0][1] * kv[0][2] * kv[0][3] * kv[0][8] * kv[0][9]):
        kind, B, gh, gw, xh, xw, yh, yw, cin, cout = prob
        if os.environ.get("TUNE_COUT") and cout != int(os.environ["TUNE_COUT"]):
            continue
        ws, nch, plan = ops.conv_query(kind, B, gh, gw, cin, cout, BF)
        if plan[4] < 0:
            continue
        taps = 4 if kind == L.CONVT_S2 else 16
        nph = 4 if kind == L.CONVT_S2 else 1
        flops = 2.0 * B * gh * gw * nph * cout * taps * cin
        t_auto = bench(prob, None)
        res = {}
        cfgs = [int(c) for c in os.environ["TUNE_CFGS"].split(",")] if os.environ.get("TUNE_CFGS") else range(NCFG)
        kss = [int(k) for k in os.environ.get("TUNE_KS", "1,2,4,8,16").split(",")]
        if os.environ.get("TUNE_CFGS"):  # a focused sweep also times the automatic plan's own config
            cfgs = sorted(set(cfgs) | {plan[4]})
        for cfg in cfgs:
            for ks in kss:
                t = bench(prob, (cfg, ks), reps=5)
                if t is not None:
                    res[(cfg, ks)] = t
        best = min(res, key=res.get)
        tot_auto += t_auto * count
        tot_best += res[best] * count
        line = (f"{names[kind]:8s} M={B * gh * gw:7d}x{nph} N={cout:4d} K={taps * cin:5d} n={count}  auto{plan[4]},{plan[2]}"
                f" {t_auto:8.1f}us {flops / t_auto / 1e6:7.1f}TF | best cfg{best[0]},ks{best[1]} {res[best]:8.1f}us "
                f"{flops / res[best] / 1e6:7.1f}TF")
        print(line, flush=True)
        out.append({"prob": prob, "count": count, "auto": [plan[4], plan[2], t_auto], "best": [best[0], best[1], res[best]],
                    "all": {f"{k[0]},{k[1]}": v for k, v in res.items()}})
    print(f"sum over one step: auto {tot_auto / 1e3:.2f} ms, best {tot_best / 1e3:.2f} ms")
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
