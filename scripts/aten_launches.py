"""Which host calls launch the non-HIP (ATen / runtime) kernels of one bench train step: torch.profiler over one
steady-state step (bs 32, bf16, the bench's schedule), every GPU kernel that is not one of ours grouped by the
Python frames that launched it.  usage: aten_launches.py [--steps-warm 3]"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps-warm", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    tr = bench.make_trainer(64, "bf16", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    B, s = 32, 256
    x = torch.rand((B, 3, s, s), generator=g, device=dev) * 2 - 1
    m = (torch.rand((B, 1, s, s), generator=g, device=dev) < 0.5).float() * 2 - 1
    y = torch.rand((B, 3, s, s), generator=g, device=dev) * 2 - 1
    for _ in range(a.steps_warm):
        tr.train_step(x, m, y)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True) as prof:
        tr.train_step(x, m, y)
        torch.cuda.synchronize()
    # CPU events that own GPU kernels (the runtime launch call, or the op itself) -> the nearest Python frames
    evs = prof.events()
    groups = collections.Counter()
    names = collections.Counter()
    for e in evs:
        ks = getattr(e, "kernels", None) or []
        for k in ks:
            n = k.name
            if ("stc::" in n or n.startswith("void stc") or "_kernel<" in n or n.endswith("_kernel")) \
                    and "at::" not in n:
                continue
            names[n[:60]] += 1
            p, stack = e, []
            while p is not None and not stack:
                stack = [f for f in (p.stack or []) if "stcgan_amd" in f or "bench" in f][:3]
                p = p.cpu_parent
            groups[(n[:40], e.name[:24], " <- ".join(stack) if stack else "?")] += 1
    print("non-HIP kernels:", sum(names.values()))
    for n, c in names.most_common():
        print(f"  {c:4d}  {n}")
    print("by launching frames:")
    for (n, op, st), c in groups.most_common(60):
        print(f"  {c:4d}  {n}  [{op}]  {st}")


if __name__ == "__main__":
    main()
