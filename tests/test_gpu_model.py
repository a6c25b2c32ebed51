"""Model-level parity of the HIP networks against the golden vectors produced by
the reference (tests/golden/*.npz) and against the CPU oracle.

Tolerances (fp32): network outputs <= 1e-4 max-abs (BASELINE.json: G2 within 1e-4
of the CPU reference); gradients within 1e-3 relative of their own max; one
train_step's post-Adam state within 1e-6 + 1e-4 relative (Adam divides by
sqrt(v), so parity of a single step is first-order in the gradient error).
"""
import numpy as np
import pytest
import torch

from fixture_init import compare, fixture_state, normal, pm_one, state_checksum, uniform
from oracle import stcgan_ref as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
NET_IN = {"G1": 3, "G2": 4, "D1": 4, "D2": 7}
NET_SEED = {"G1": 11, "G2": 12, "D1": 13, "D2": 14}


def make_net(name, ngf, family="one", dtype="fp32"):
    from stcgan_amd import networks
    if name == "G1":
        net = networks.get_generator(3, 1, ngf=ngf)
    elif name == "G2":
        net = networks.get_generator(4, 3, ngf=ngf)
    else:
        net = networks.get_discriminator(NET_IN[name], ndf=ngf, n_layers=3, use_sigmoid=False)
    st = fixture_state(net.state_dict(), NET_SEED[name], family)
    net.load_state_dict(st)
    net.to(DEV)
    net.set_compute_dtype(dtype)
    return net, st


def test_state_dict_keys_match_reference():
    for name in ["G1", "G2", "D1", "D2"]:
        from stcgan_amd import networks
        net = (networks.get_generator(3 if name == "G1" else 4, 1 if name == "G1" else 3, ngf=64)
               if name.startswith("G") else networks.get_discriminator(NET_IN[name], ndf=64))
        tmpl = (ref.generator_state_template(3 if name == "G1" else 4, 1 if name == "G1" else 3, 64)
                if name.startswith("G") else ref.discriminator_state_template(NET_IN[name], 64))
        sd = net.state_dict()
        assert list(sd.keys()) == list(tmpl.keys())
        for k in sd:
            assert tuple(sd[k].shape) == tuple(tmpl[k].shape), k


@pytest.mark.parametrize("name", ["G1", "G2", "D1", "D2"])
def test_nets_ngf8_vs_golden(golden, name):
    d = golden("nets_ngf8.npz")
    bs, hw = int(d["meta/bs"]), int(d["meta/hw"])
    net, st = make_net(name, 8)
    assert abs(state_checksum(st) - float(d[f"{name}/checksum"])) < 1e-6
    # input seed chosen by the generator so no deep-level activation input sits within 1e-5
    # of zero (a ReLU decision there is fp32-rounding-sensitive; see make_goldens.pick_input_seed)
    x = uniform((bs, NET_IN[name], hw, hw), int(d[f"{name}/x_seed"])).to(DEV).requires_grad_(True)
    net.train()
    out = net(x)
    r = normal(tuple(out.shape), 200 + NET_SEED[name]).to(DEV)
    (out * r).sum().backward()
    torch.cuda.synchronize()
    compare(d, f"{name}/train_out", out.detach().cpu(), atol=1e-4)
    compare(d, f"{name}/input_grad", x.grad.cpu(), atol=2e-5, rtol=2e-3)
    for k, p in net.named_parameters():
        g = d.get(f"{name}/grad/{k}")
        scale = float(np.abs(g).max()) if g is not None else 1.0
        compare(d, f"{name}/grad/{k}", p.grad.cpu(), atol=2e-4 * scale + 1e-6, rtol=2e-3)
    for k, b in net.named_buffers():
        compare(d, f"{name}/buf_after_train/{k}", b.cpu(), atol=1e-5, rtol=1e-4)
    net.load_state_dict(st)
    net.eval()
    with torch.no_grad():
        compare(d, f"{name}/eval_out", net(x.detach()).cpu(), atol=1e-4)


@pytest.mark.parametrize("name", ["G1", "G2"])
def test_generator_ngf64_vs_golden(golden, name):
    """Full-width generator at 256x256: the BASELINE.json 1e-4 max-abs criterion."""
    d = golden("g_ngf64.npz")
    net, st = make_net(name, 64)
    assert abs(state_checksum(st) - float(d[f"{name}/checksum"])) < 1e-6 * float(d[f"{name}/checksum"])
    x = uniform((1, NET_IN[name], 256, 256), 300 + NET_SEED[name]).to(DEV)
    net.train()
    with torch.no_grad():
        y = net(x).cpu().numpy()
    err = float(np.abs(y - d[f"{name}/train_out"]).max())
    assert err <= 1e-4, f"{name} train-mode max-abs {err:.3e}"
    net.load_state_dict(st)
    net.eval()
    with torch.no_grad():
        y = net(x).cpu().numpy()
    err = float(np.abs(y - d[f"{name}/eval_out"]).max())
    assert err <= 1e-4, f"{name} eval-mode max-abs {err:.3e}"


def istd_input(d):
    f = d["shadow_bgr_u8"].astype(np.float32) / 255
    f = (f - 0.5) * 2
    return torch.from_numpy(np.ascontiguousarray(f.transpose(2, 0, 1)))[None]


@pytest.mark.parametrize("train", [False, True])
def test_istd_480x640_vs_golden(golden, train):
    """Native-resolution ISTD pair through G1 -> G2 (odd intermediate sizes 15x20 and 4x5)."""
    d = golden("istd_114_5.npz")
    x = istd_input(d).to(DEV)
    g1, s1 = make_net("G1", 64)
    g2, s2 = make_net("G2", 64)
    g1.train(train)
    g2.train(train)
    with torch.no_grad():
        m = g1(x)
        y = g2([x, m])
    key = "full_train" if train else "full"
    em = float(np.abs(m.cpu().numpy() - d[f"{key}/m_pred"]).max())
    ey = float(np.abs(y.cpu().numpy() - d[f"{key}/y_pred"]).max())
    assert em <= 1e-4 and ey <= 1e-4, (em, ey)


def test_istd_crop_vs_golden(golden):
    d = golden("istd_114_5.npz")
    r0, c0 = (int(v) for v in d["crop/r0c0"])
    x = istd_input(d)[:, :, r0:r0 + 256, c0:c0 + 256].contiguous().to(DEV)
    g1, _ = make_net("G1", 64)
    g2, _ = make_net("G2", 64)
    g1.eval()
    g2.eval()
    with torch.no_grad():
        m = g1(x)
        y = g2(torch.cat((x, m), 1))
    assert float(np.abs(m.cpu().numpy() - d["crop/m_pred"]).max()) <= 1e-4
    assert float(np.abs(y.cpu().numpy() - d["crop/y_pred"]).max()) <= 1e-4


def _trainer(ngf, loss_type="normal", dtype="fp32"):
    import types
    from stcgan_amd.stcgan import STCGAN
    args = types.SimpleNamespace(devices=["cuda"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                                 D_loss_fn="standard", D_loss_type=loss_type, ngf=ngf, dtype=dtype,
                                 load_weights_g1=None, load_weights_g2=None, load_weights_d1=None,
                                 load_weights_d2=None)
    tr = STCGAN(args)
    for name in ["G1", "G2", "D1", "D2"]:
        net = getattr(tr, name)
        net.load_state_dict(fixture_state(net.state_dict(), NET_SEED[name], "ref"))
    return tr


def _batches(n, bs, hw, seed):
    out = []
    for i in range(n):
        s = seed + 10 * i
        out.append(([], uniform((bs, 3, hw, hw), s), pm_one((bs, 1, hw, hw), s + 1), uniform((bs, 3, hw, hw), s + 2)))
    return out


@pytest.mark.parametrize("loss_type", ["one_iter", "normal", "rel", "rel_avg"])
def test_run_epoch_vs_golden(golden, loss_type):
    """The reference's run_epoch (STCGAN/stcgan.py:186-330) at ngf=8: losses and post-Adam state."""
    d = golden("run_epoch_ngf8.npz")
    ngf, bs, hw = int(d["meta/ngf"]), int(d["meta/bs"]), int(d["meta/hw"])
    one = loss_type == "one_iter"
    batches = _batches(int(d["meta/n_iter"]), bs, hw, int(d["meta/batch_seed"]))
    if one:
        batches = batches[:1]
    tr = _trainer(ngf, "normal" if one else loss_type)
    tr.train_loader = batches
    tr.valid_loader = batches
    # Tolerances.  With the reference init (BN gamma ~ N(0, 0.02)) many gradients are
    # tiny sums with heavy cancellation; Adam's first step is lr*g/(|g|+eps), so for
    # |g| ~ eps a relative gradient difference moves the update by up to ~lr/4:
    # one-iteration state is checked to 0.2*lr_G = 1e-5 (gradients themselves are
    # checked tightly in test_nets_ngf8_vs_golden).  Two iterations: Adam's second
    # step amplifies further (tests/test_oracle_golden.py::test_oracle_run_epoch), so
    # state is checked to 1 lr step and the logged losses / D outputs (means of values
    # ~1e-3 that depend on those updates) to 1e-4 absolute.
    m_atol = 2e-5 if one else 1e-4
    meas = tr.run_epoch(training=True)
    for grp, vals in meas.items():
        for k, v in vals.items():
            want = float(d[f"{loss_type}/measures/{grp}/{k}"])
            assert abs(v - want) <= m_atol + 2e-4 * abs(want), (grp, k, v, want)
    for n in ["G1", "G2", "D1", "D2"]:
        for k, v in getattr(tr, n).state_dict().items():
            compare(d, f"{loss_type}/state/{n}/{k}", v.cpu(), atol=1e-5 if one else 5e-5, rtol=1e-4)
    meas = tr.run_epoch(training=False)
    for grp, vals in meas.items():
        for k, v in vals.items():
            want = float(d[f"{loss_type}/valid_measures/{grp}/{k}"])
            assert abs(v - want) <= m_atol + 2e-4 * abs(want), (grp, k, v, want)


def test_bf16_generator_vs_oracle():
    """bf16 operands / fp32 accumulation: G2 within 2e-2 max-abs of the fp32 oracle (stated bf16 tolerance)."""
    net, st = make_net("G2", 64, dtype="bf16")
    x = uniform((2, 4, 256, 256), 777)
    net.train()
    with torch.no_grad():
        y = net(x.to(DEV)).cpu()
        yr = ref.generator_forward({k: v.clone() for k, v in st.items()}, x, True)
    err = float((y - yr).abs().max())
    assert err <= 2e-2, f"bf16 G2 max-abs {err:.3e}"


def test_bf16_train_step_runs_and_tracks_fp32():
    """A bf16 train step at ngf=8: losses within 2e-2 relative of the fp32 HIP step."""
    batches = _batches(1, 2, 256, 500)
    res = {}
    for dt in ["fp32", "bf16"]:
        tr = _trainer(8, dtype=dt)
        tr.train_loader = batches
        res[dt] = tr.run_epoch(training=True)["Loss"]
    for k in ["G", "D", "data1", "data2"]:
        a, b = res["fp32"][k], res["bf16"][k]
        assert abs(a - b) <= 2e-2 * abs(a) + 1e-4, (k, a, b)
