"""K bf16 bs=32 256^2 train steps (the bench workload) and nothing else: the command profiled by
scripts/gpu_steps.sh, so per-step kernel totals are the rocprof totals / (K + W)."""
import argparse
import json
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import engine  # noqa: E402
from stcgan_amd.stcgan import STCGAN  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=4)
ap.add_argument("--warmup", type=int, default=2)
ap.add_argument("--dtype", default="bf16")
ap.add_argument("--streams", type=int, default=1)
ap.add_argument("--fused", type=int, default=1)
ap.add_argument("--host-sleep-us", type=int, default=0, help="extra host time per step (host-boundness probe)")
ap.add_argument("--repeat", type=int, default=1)
ap.add_argument("--wgrad-overlap", type=int, default=1)
ap.add_argument("--ab", default="", help="comma list of wgrad-overlap settings cycled per repeat (same process)")
ap.add_argument("--ab-attr", default="", help="name=v1,v2: trainer attribute (int) cycled per repeat (same process)")
ap.add_argument("--ab-plans", default="", help="JSON list of {name, conv: [[key..., cfg, ks]], wgrad: [[key..., cfg, "
                "splits]]} plan-override settings cycled per repeat (same process)")
args = ap.parse_args()
engine.WGRAD_OVERLAP = args.wgrad_overlap > 0
if args.wgrad_overlap > 1:
    engine.WGRAD_OVERLAP_MAX_PIX = args.wgrad_overlap
a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                          D_loss_fn="standard", D_loss_type="normal", ngf=64, dtype=args.dtype, load_weights_g1=None,
                          load_weights_g2=None, load_weights_d1=None, load_weights_d2=None,
                          streams=bool(args.streams), fused_objectives=bool(args.fused))
torch.manual_seed(1234)
tr = STCGAN(a)
import stcgan_amd.stcgan as _st  # noqa: E402
tr.set_early = lambda v: setattr(_st, "EARLY_D_BACKWARD", int(v))  # (--ab-attr early=0,1,2)
tr.set_late = lambda v: setattr(_st, "LATE_STATS_CALLS", bool(v))  # (--ab-attr late=0,1)
if args.host_sleep_us:
    _ts = tr.train_step

    def _slow(*aa, **kk):
        t_end = time.perf_counter() + args.host_sleep_us * 1e-6
        while time.perf_counter() < t_end:
            pass
        return _ts(*aa, **kk)
    tr.train_step = _slow
dev = torch.device("cuda", 0)
B = 32
x = torch.rand((B, 3, 256, 256), device=dev) * 2 - 1
m = (torch.rand((B, 1, 256, 256), device=dev) < 0.5).float() * 2 - 1
y = torch.rand((B, 3, 256, 256), device=dev) * 2 - 1
for _ in range(args.warmup):
    tr.train_step(x, m, y)
torch.cuda.synchronize()
ab = [int(v) for v in args.ab.split(",")] if args.ab else None
plans = json.loads(args.ab_plans) if args.ab_plans else None
res = {}
attr = None
if args.ab_attr:
    an, av = args.ab_attr.split("=")
    attr = (an, [int(v) for v in av.split(",")])
for rep in range(args.repeat):
    if attr:
        v = attr[1][rep % len(attr[1])]
        setter = getattr(tr, "set_" + attr[0], None)
        if setter is not None:
            setter(v)
        else:
            setattr(tr, attr[0], type(getattr(tr, attr[0]))(v))
        args.wgrad_overlap = f"{attr[0]}={v}"
        for _ in range(2):
            tr.train_step(x, m, y)
        torch.cuda.synchronize()
    if plans:
        from stcgan_amd import ops
        pl = plans[rep % len(plans)]
        ops.FORCE_CONV.clear()
        ops.FORCE_WGRAD.clear()
        for e in pl.get("conv", []):
            ops.FORCE_CONV[tuple(e[:6])] = tuple(e[6:8])
        for e in pl.get("wgrad", []):
            ops.FORCE_WGRAD[tuple(e[:5])] = tuple(e[5:7])
        args.wgrad_overlap = pl["name"]
        for _ in range(2):
            tr.train_step(x, m, y)
        torch.cuda.synchronize()
    if ab:
        o = ab[rep % len(ab)]
        engine.WGRAD_OVERLAP = o > 0
        engine.WGRAD_OVERLAP_MAX_PIX = o if o > 1 else 1 << 30
        args.wgrad_overlap = o
        for _ in range(2):
            tr.train_step(x, m, y)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.train_step(x, m, y)
    torch.cuda.synchronize()
    print(f"{(time.perf_counter() - t0) / args.steps * 1e3:.3f} ms/step  mem {torch.cuda.memory_allocated() / 2**30:.2f} GiB "
          f"reserved {torch.cuda.memory_reserved() / 2**30:.2f} GiB ({args.steps} steps, streams={args.streams}, "
          f"fused={args.fused}, wgrad_overlap={args.wgrad_overlap})", flush=True)
    res.setdefault(args.wgrad_overlap, []).append((time.perf_counter() - t0) / args.steps * 1e3)
if ab or plans or attr:
    for k, v in res.items():
        print(f"wgrad_overlap={k}: median {sorted(v)[len(v) // 2]:.3f} ms/step over {len(v)}", flush=True)
