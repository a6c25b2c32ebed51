"""When do the gradient buckets become ready during the backward, and how much all-reduce would stay exposed at
world 8?  One bench-config train step (bs 32, bf16, 256x256) on one GPU with BucketExchange tracing (every
parameter's gradient-ready event, on the stream that wrote it, and each network's finish), then a simulation of
the RCCL ring all-reduce of the same buckets at world W on one communicator (collectives run one after another
in ready order): cost = alpha + 2 (W - 1) / W * bytes / busbw.  Prints per network: gradient bytes, the window
from its first gradient to its backward's end, the exposed time after it for each bucket size and bus bandwidth,
without and with overlap_optim (each bucket's share of the measured optimiser update right after its all-reduce;
reported as the time past the one-GPU step's backward + update).
usage: exchange_timeline.py [--world 8] [--alpha-us 25]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from stcgan_amd import parallel  # noqa: E402

NETS = ("D1", "D2", "G1", "G2")


def buckets_of(flat, bucket_mb):
    """Bucket boundaries as BucketExchange cuts them (reverse module order): [(param ids, bytes)]."""
    lim = max(1, int(bucket_mb * (1 << 20) // 4))
    out, cur, n = [], [], 0
    for p in reversed(flat.params):
        cur.append(id(p))
        n += p.numel()
        if n >= lim:
            out.append((cur, 4 * n))
            cur, n = [], 0
    if cur:
        out.append((cur, 4 * n))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--alpha-us", type=float, default=25.0)
    a = ap.parse_args()
    torch.manual_seed(1234)
    tr = bench.make_trainer(64, "bf16", 0)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    x = torch.rand((32, 3, 256, 256), generator=g, device=dev) * 2 - 1
    m = (torch.rand((32, 1, 256, 256), generator=g, device=dev) < 0.5).float() * 2 - 1
    y = torch.rand((32, 3, 256, 256), generator=g, device=dev) * 2 - 1
    for net in (tr.G1, tr.G2, tr.D1, tr.D2):
        net.train()
    for _ in range(3):
        tr.train_step(x, m, y)
    torch.cuda.synchronize()
    for n in NETS:
        getattr(tr, n).grad_exchange.trace = []
    t0 = torch.cuda.Event(enable_timing=True)
    t0.record()
    tr.train_step(x, m, y)
    t1 = torch.cuda.Event(enable_timing=True)
    t1.record()
    torch.cuda.synchronize()
    step_ms = t0.elapsed_time(t1)
    # the optimiser updates alone (one more step() each on the same gradients: timing only)
    upd = {}
    for phase, o in (("D", tr.optim_D), ("G", tr.optim_G)):
        u0, u1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        u0.record()
        o.step()
        u1.record()
        torch.cuda.synchronize()
        upd[phase] = u0.elapsed_time(u1)
    res = {"step_ms": round(step_ms, 3), "world": a.world, "alpha_us": a.alpha_us, "update_ms": upd, "nets": {}}
    ready, fin, flats = {}, {}, {}
    for n in NETS:
        ex = getattr(tr, n).grad_exchange
        flats[n] = ex.flat
        for ids, ev in ex.trace:
            t = t0.elapsed_time(ev)
            if ids == "finish":
                fin[n] = t
                continue
            for i in ids:  # the last report counts (the discriminators report twice in the D step)
                ready[i] = max(ready.get(i, 0.0), t)
        ex.trace = None
    # the D step's exchange: D1 + D2 buckets before optim_D.step; the G step's: G1 + G2 before optim_G.step
    sims = {}
    for phase, nets in (("D", ("D1", "D2")), ("G", ("G1", "G2"))):
        end = max(fin[n] for n in nets)
        first = min(ready[id(p)] for n in nets for p in flats[n].params)
        nbytes = sum(4 * flats[n].numel for n in nets)
        sims[phase] = {"grad_MB": round(nbytes / 1e6, 1), "first_ready_ms": round(first, 3),
                       "backward_end_ms": round(end, 3), "window_ms": round(end - first, 3), "exposed_ms": {},
                       "exposed_overlap_optim_ms": {}}
        for mb in (4, 8, 16, 32, 64, 128):
            bks = []
            for n in nets:
                for ids, b in buckets_of(flats[n], mb):
                    bks.append((max(ready[i] for i in ids), b))
            bks.sort()
            for bw in (150, 300, 600):
                t = u = 0.0
                for r, b in bks:
                    t = max(t, r) + a.alpha_us * 1e-3 + 2 * (a.world - 1) / a.world * b / (bw * 1e9) * 1e3
                    # overlap_optim: the bucket's share of the update right after its all-reduce, one bucket at a
                    # time on the optimiser stream
                    u = max(u, t) + upd[phase] * b / nbytes
                sims[phase]["exposed_ms"][f"{mb}MB@{bw}GB/s"] = round(max(0.0, t - end), 3)
                # time past the eager step (whose update follows its backward): (update done) - (end + update)
                sims[phase]["exposed_overlap_optim_ms"][f"{mb}MB@{bw}GB/s"] = round(u - end - upd[phase], 3)
    res["phases"] = sims
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
