"""Adam + operand-repack launch variants (STC_ADAM_VARIANT: bit 0 XCD-grouped tiles, bit 1 streaming stores) on
the generators' real parameter set (ngf=64, bf16 operands): interleaved timings of optim_G.step(); with
argument "hash", a state hash after three train steps under the variant in the environment (bit-identity
across variants is compared between processes)."""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd.stcgan import STCGAN  # noqa: E402

a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                          D_loss_fn="standard", D_loss_type="normal", ngf=64, dtype="bf16", load_weights_g1=None,
                          load_weights_g2=None, load_weights_d1=None, load_weights_d2=None)
torch.manual_seed(0)
tr = STCGAN(a)
dev = torch.device("cuda", 0)
B = 32
x = torch.rand((B, 3, 256, 256), device=dev) * 2 - 1
m = (torch.rand((B, 1, 256, 256), device=dev) < 0.5).float() * 2 - 1
y = torch.rand((B, 3, 256, 256), device=dev) * 2 - 1
for _ in range(2):
    tr.train_step(x, m, y)
torch.cuda.synchronize()
opt = tr.optim_G
nets = (tr.G1, tr.G2)


def _tensors(o, out):
    if torch.is_tensor(o):
        if o.is_cuda:
            out.append(o)
    elif isinstance(o, dict):
        for k in sorted(o, key=str):
            _tensors(o[k], out)
    elif isinstance(o, (list, tuple)):
        for v in o:
            _tensors(v, out)
    return out


def live():
    t = [p.detach() for g in opt.param_groups for p in g["params"]]
    for st in opt.state.values():
        _tensors(st, t)
    for net in nets:
        _tensors(net._pack_cache, t)
    return t


VARIANTS = [int(v) for v in os.environ.get("AB_VARIANTS", "0,1,2,3").split(",")]


def run(variant, reps=10):
    os.environ["STC_ADAM_VARIANT"] = str(variant)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for it in range(reps + 2):
        if it == 2:
            e0.record()
        opt.step()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


if len(sys.argv) > 1 and sys.argv[1] == "hash":
    # bit-identity across variants: a third train step under the variant in the environment, then a hash of
    # the parameters, the Adam state and both generators' outputs (these read the packed operands); the training
    # step is deterministic run to run
    tr.train_step(x, m, y)
    torch.cuda.synchronize()
    import hashlib
    def digest(ts):
        h = hashlib.sha256()
        for t in ts:
            h.update(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes())
        return h.hexdigest()[:12]

    params = [p for g in opt.param_groups for p in g["params"]]
    cats = {"params": params,
            "exp_avg": [opt.state[p]["exp_avg"] for p in params],
            "exp_avg_sq": [opt.state[p]["exp_avg_sq"] for p in params],
            "G1/G2 outputs": [tr.G1(x).float(), tr.G2([x, tr.G1(x)]).float()]}
    print("variant", os.environ.get("STC_ADAM_VARIANT", "0"), "state hash",
          "  ".join(f"{k} {digest(v)}" for k, v in cats.items()))
    sys.exit(0)
for _ in range(3):
    print("  ".join(f"v{v} {run(v):8.1f} us" for v in VARIANTS), flush=True)
