"""Single-process check that the side-stream step is reproducible and equal to the serial one:
bf16 ngf=16 bs=4 two train steps, every gradient of both steps and the final state compared."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402
from dist_diag import batches, trainer, NETS  # noqa: E402


def run(streams):
    tr = trainer(streams, False)
    grads = []
    for (x, m, y) in batches():
        for opt in (tr.optim_D, tr.optim_G):
            st0 = opt.step

            def cap(st0=st0, opt=opt):
                grads.append({f"{'D' if opt is tr.optim_D else 'G'}.{i}.{tuple(p.shape)}":
                              (p.grad.detach().cpu().clone() if p.grad is not None else None)
                              for i, p in enumerate([q for g in opt.param_groups for q in g["params"]])})
                st0()
            opt.step = cap
        tr.train_step(x.cuda(), m.cuda(), y.cuda())
        for opt in (tr.optim_D, tr.optim_G):
            del opt.step
    torch.cuda.synchronize()
    return grads, {n: {k: v.cpu() for k, v in getattr(tr, n).state_dict().items()} for n in NETS}


def cmp(a, b, tag):
    bad = []
    for i, (ga, gb) in enumerate(zip(a[0], b[0])):
        for k in ga:
            if ga[k] is None or gb[k] is None:
                if (ga[k] is None) != (gb[k] is None):
                    bad.append(f"grad set {i} {k} None mismatch")
                continue
            if not torch.equal(ga[k], gb[k]):
                bad.append(f"grad set {i} {k} {float((ga[k] - gb[k]).abs().max()):.3e}")
    for n in NETS:
        for k in a[1][n]:
            if not torch.equal(a[1][n][k], b[1][n][k]):
                bad.append(f"state {n}.{k}")
    print(f"{tag}: {len(bad)} mismatches", *bad[:10], sep="\n  ", flush=True)


off = run(False)
for rep in range(4):
    on = run(True)
    cmp(on, off, f"streams on (run {rep}) vs off")
off2 = run(False)
cmp(off2, off, "streams off vs off")


def run_nosync(streams, nsteps=2):
    tr = trainer(streams, False)
    bs = batches()
    for i in range(nsteps):
        x, m, y = bs[i % 2]
        tr.train_step(x.cuda(), m.cuda(), y.cuda())
    torch.cuda.synchronize()
    return [], {n: {k: v.cpu() for k, v in getattr(tr, n).state_dict().items()} for n in NETS}


for ns in (2, 3):
    ref = run_nosync(False, ns)
    for rep in range(3):
        cmp(run_nosync(True, ns), ref, f"no host sync, {ns} steps: streams on (run {rep}) vs off")
