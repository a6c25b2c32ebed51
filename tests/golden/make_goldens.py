#!/usr/bin/env python
"""Generate the golden vectors under tests/golden/ by running the REFERENCE code.

TEST INFRASTRUCTURE ONLY -- runs in the build container, where the reference is
mounted read-only at /root/reference.  It is never run on the GPU box and never
shipped: only its outputs (the .npz fixtures next to this file) are committed.

What is imported:
  * STCGAN/networks.py     -- directly (needs only torch)
  * STCGAN/loss.py, STCGAN/stcgan.py -- with stub modules for cv2, torchvision,
    h5py and torch.utils.tensorboard (none of them is on the computed path);
    STCGAN.__init__ cannot run here (ReduceLROnPlateau(verbose=True) raises on
    torch 2.10 and the loaders need cv2 + ISTD dirs), so the object is built
    with object.__new__ and the reference's own run_epoch() is called on a
    list of synthetic batches.
  * src/models/stcgan_g.py -- the odd-size-safe generator used for 480x640.
The ISTD triplet 114-5 (color_adjustment_code/*.png, 640x480) is read with PIL
and flipped RGB->BGR to match cv.imread (STCGAN/dataset.py:96-112).

Usage:  python tests/golden/make_goldens.py   (writes tests/golden/*.npz)
"""
import logging
import os
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True  # the reference tree is read-only
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from fixture_init import fixture_state, normal, pm_one, put, state_checksum, uniform  # noqa: E402

REF = "/root/reference"


def _install_stubs():
    for name in ["cv2", "torchvision", "torchvision.models", "h5py"]:
        mod = types.ModuleType(name)
        sys.modules[name] = mod
    sys.modules["torchvision"].models = sys.modules["torchvision.models"]
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:  # never used on the computed path
        def __init__(self, *a, **k):
            pass

    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb


def import_reference():
    _install_stubs()
    sys.path.insert(0, os.path.join(REF, "STCGAN"))
    import networks  # noqa
    import loss  # noqa
    import stcgan  # noqa
    sys.path.insert(0, REF)
    from src.models import stcgan_g  # noqa
    return networks, loss, stcgan, stcgan_g


def net_specs(networks, ngf):
    return {
        "G1": lambda: networks.get_generator(3, 1, ngf=ngf),
        "G2": lambda: networks.get_generator(4, 3, ngf=ngf),
        "D1": lambda: networks.get_discriminator(4, ndf=ngf, n_layers=3, use_sigmoid=False),
        "D2": lambda: networks.get_discriminator(7, ndf=ngf, n_layers=3, use_sigmoid=False),
    }


NET_IN = {"G1": 3, "G2": 4, "D1": 4, "D2": 7}
NET_SEED = {"G1": 11, "G2": 12, "D1": 13, "D2": 14}


def activation_margin(net, x, max_numel):
    """Smallest |input| of any ReLU/LeakyReLU whose input has <= max_numel elements (deep levels).
    A value within fp32 rounding of 0 there can take the other branch on another
    summation order and legitimately change every gradient below it."""
    mins = []

    def hook(mod, inp):
        t = inp[0]
        if t.numel() <= max_numel:
            mins.append(float(t.detach().abs().min()))

    hs = [m.register_forward_pre_hook(hook) for m in net.modules()
          if isinstance(m, (torch.nn.ReLU, torch.nn.LeakyReLU))]
    with torch.no_grad():
        net.train()
        net(x)
    for h in hs:
        h.remove()
    return min(mins) if mins else float("inf")


def pick_input_seed(net, st, shape, base, max_numel, margin=1e-5):
    """First input seed (base, base+1000, ...) whose deep-level activation inputs all keep
    |v| >= margin (evaluated on a fresh copy of the fixture state)."""
    for trial in range(50):
        seed = base + 1000 * trial
        net.load_state_dict(st)
        if activation_margin(net, uniform(shape, seed), max_numel) >= margin:
            net.load_state_dict(st)
            return seed
    raise RuntimeError("no well-conditioned input seed found")


def gen_nets(networks, ngf=8, bs=2, hw=256):
    """Per-network forward (train/eval) and backward goldens at reduced width, full depth."""
    d = {}
    for name, ctor in net_specs(networks, ngf).items():
        net = ctor()
        st = fixture_state(net.state_dict(), NET_SEED[name], "one")
        net.load_state_dict(st)
        d[f"{name}/checksum"] = np.array(state_checksum(st))
        shape = (bs, NET_IN[name], hw, hw)
        # deep levels = activations at <= 16x16 for the whole batch and the widest channel count
        xseed = pick_input_seed(net, st, shape, 100 + NET_SEED[name], bs * 16 * ngf * 16 * 16)
        d[f"{name}/x_seed"] = np.array(xseed)
        x = uniform(shape, xseed)
        # train mode forward + backward of sum(out * R)
        net.train()
        xg = x.clone().requires_grad_(True)
        out = net(xg)
        r = normal(tuple(out.shape), 200 + NET_SEED[name])
        (out * r).sum().backward()
        put(d, f"{name}/train_out", out)
        put(d, f"{name}/input_grad", xg.grad)
        for k, p in net.named_parameters():
            put(d, f"{name}/grad/{k}", p.grad)
        for k, b in net.named_buffers():
            put(d, f"{name}/buf_after_train/{k}", b)
        # eval mode with the fixture running stats
        net.load_state_dict(st)
        net.eval()
        with torch.no_grad():
            put(d, f"{name}/eval_out", net(x))
    d["meta/ngf"] = np.array(ngf)
    d["meta/bs"] = np.array(bs)
    d["meta/hw"] = np.array(hw)
    return d


def make_trainer(networks, loss, stcgan, ngf, loss_type, batches):
    """Reference STCGAN object without __init__."""
    t = object.__new__(stcgan.STCGAN)
    t.logger = logging.getLogger("golden")
    t.device = torch.device("cpu")
    nets = {}
    for name, ctor in net_specs(networks, ngf).items():
        net = ctor()
        net.load_state_dict(fixture_state(net.state_dict(), NET_SEED[name], "ref"))
        nets[name] = net
    t.G1, t.G2, t.D1, t.D2 = nets["G1"], nets["G2"], nets["D1"], nets["D2"]
    # hyper-parameters of STCGAN/main.py:125-132,218-226 and STCGAN/stcgan.py:60-71
    t.optim_G = torch.optim.Adam(list(t.G1.parameters()) + list(t.G2.parameters()),
                                 lr=0.00005, betas=(0.5, 0.999))
    t.optim_D = torch.optim.Adam(list(t.D1.parameters()) + list(t.D2.parameters()),
                                 lr=0.00002, betas=(0.5, 0.999))
    t.decay_G = torch.optim.lr_scheduler.ReduceLROnPlateau(t.optim_G, cooldown=10, min_lr=1e-7, factor=0.8)
    t.decay_D = torch.optim.lr_scheduler.ReduceLROnPlateau(t.optim_D, cooldown=10, min_lr=1e-7, factor=0.8)
    t.d_loss_fn = "standard"
    t.d_loss_type = loss_type
    t.adv_loss = loss.AdversarialLoss(ls=False)  # the "leastsqure" typo: ls is always False
    t.data_loss = loss.DataLoss()
    t.lambda1, t.lambda2, t.lambda3 = 5, 0.1, 0.1
    t.adapt = False
    t.train_loader = batches
    t.valid_loader = batches
    return t


def synth_batches(n, bs, hw, seed):
    out = []
    for i in range(n):
        s = seed + 10 * i
        x = uniform((bs, 3, hw, hw), s)
        m = pm_one((bs, 1, hw, hw), s + 1)
        y = uniform((bs, 3, hw, hw), s + 2)
        out.append(([f"img{i}_{j}" for j in range(bs)], x, m, y))
    return out


def gen_run_epoch(networks, loss, stcgan, ngf=8, bs=2, hw=256, n_iter=2):
    d = {}
    batches = synth_batches(n_iter, bs, hw, 500)
    # "one_iter": a single iteration, full state tensors (tight parity: no Adam
    # amplification yet); 2-iteration runs for every loss type as summaries.
    for loss_type in ["one_iter", "normal", "rel", "rel_avg"]:
        lt = "normal" if loss_type == "one_iter" else loss_type
        bt = batches[:1] if loss_type == "one_iter" else batches
        t = make_trainer(networks, loss, stcgan, ngf, lt, bt)
        meas = t.run_epoch(training=True)
        for grp, vals in meas.items():
            for k, v in vals.items():
                d[f"{loss_type}/measures/{grp}/{k}"] = np.array(float(v))
        for name in ["G1", "G2", "D1", "D2"]:
            for k, v in getattr(t, name).state_dict().items():
                # full tensors for the default loss type, summaries for the variants
                put(d, f"{loss_type}/state/{name}/{k}", v,
                    limit=None if loss_type == "one_iter" else 4096)
        # a validation epoch afterwards (eval-mode BN, no optimiser step)
        meas = t.run_epoch(training=False)
        for grp, vals in meas.items():
            for k, v in vals.items():
                d[f"{loss_type}/valid_measures/{grp}/{k}"] = np.array(float(v))
    d["meta/ngf"] = np.array(ngf)
    d["meta/bs"] = np.array(bs)
    d["meta/hw"] = np.array(hw)
    d["meta/n_iter"] = np.array(n_iter)
    d["meta/batch_seed"] = np.array(500)
    return d


def gen_ngf64(networks):
    d = {}
    for name in ["G1", "G2"]:
        net = net_specs(networks, 64)[name]()
        st = fixture_state(net.state_dict(), NET_SEED[name], "one")
        net.load_state_dict(st)
        d[f"{name}/checksum"] = np.array(state_checksum(st))
        x = uniform((1, NET_IN[name], 256, 256), 300 + NET_SEED[name])
        net.train()
        with torch.no_grad():
            d[f"{name}/train_out"] = net(x).numpy()
        net.load_state_dict(st)
        net.eval()
        with torch.no_grad():
            d[f"{name}/eval_out"] = net(x).numpy()
    return d


def gen_ngf64_grad(networks, loss, bs=2, hw=256):
    """Full-width (ngf=64) G1 -> G2 forward + backward through the reference's DataLoss
    (data1 + 5 * data2, STCGAN/stcgan.py:292-303 without the adversarial terms): outputs,
    every parameter gradient and the input gradient as summaries (sum, |sum|, sum of squares,
    512 fixed samples), BN buffers after the train-mode forward in full."""
    d = {}
    g1 = net_specs(networks, 64)["G1"]()
    g2 = net_specs(networks, 64)["G2"]()
    s1 = fixture_state(g1.state_dict(), NET_SEED["G1"], "one")
    s2 = fixture_state(g2.state_dict(), NET_SEED["G2"], "one")
    g1.load_state_dict(s1)
    g2.load_state_dict(s2)
    d["G1/checksum"] = np.array(state_checksum(s1))
    d["G2/checksum"] = np.array(state_checksum(s2))
    # deep levels (<= 8x8 at ngf=64 widths) kept away from the ReLU kink, as for the ngf=8 goldens
    xseed = pick_input_seed(g1, s1, (bs, 3, hw, hw), 900, bs * 512 * 8 * 8)
    d["meta/x_seed"] = np.array(xseed)
    x = uniform((bs, 3, hw, hw), xseed).requires_grad_(True)
    m = pm_one((bs, 1, hw, hw), xseed + 1)
    y = uniform((bs, 3, hw, hw), xseed + 2)
    g1.train()
    g2.train()
    dl = loss.DataLoss()
    m_pred = g1(x)
    y_pred = g2(torch.cat((x, m_pred), dim=1))
    data1 = dl(m_pred, m)
    data2 = dl(y_pred, y)
    total = data1 + 5 * data2
    total.backward()
    d["data1"] = np.array(float(data1))
    d["data2"] = np.array(float(data2))
    put(d, "m_pred", m_pred)
    put(d, "y_pred", y_pred)
    put(d, "input_grad", x.grad)
    for name, net in (("G1", g1), ("G2", g2)):
        for k, p in net.named_parameters():
            put(d, f"{name}/grad/{k}", p.grad)
        for k, b in net.named_buffers():
            put(d, f"{name}/buf_after_train/{k}", b)
    d["meta/bs"] = np.array(bs)
    d["meta/hw"] = np.array(hw)
    return d


def load_istd():
    from PIL import Image
    base = os.path.join(REF, "color_adjustment_code")
    shadow = np.array(Image.open(os.path.join(base, "114-5_shadow.png")).convert("RGB"))[:, :, ::-1]
    mask = np.array(Image.open(os.path.join(base, "114-5_shadow_mask.png")).convert("L"))
    free = np.array(Image.open(os.path.join(base, "114-5_shadow_free_original.png")).convert("RGB"))[:, :, ::-1]
    return np.ascontiguousarray(shadow), np.ascontiguousarray(mask), np.ascontiguousarray(free)


def to_input(u8):
    """uint2float (STCGAN/utils.py:58-60) then (v-0.5)*2 (STCGAN/dataset.py:124-126), HWC->NCHW."""
    f = u8.astype(np.float32) / 255
    f = (f - 0.5) * 2
    if f.ndim == 2:
        f = f[:, :, None]
    return torch.from_numpy(np.ascontiguousarray(f.transpose(2, 0, 1)))[None]


def gen_istd(networks, stcgan_g):
    d = {}
    shadow, mask, free = load_istd()
    d["shadow_bgr_u8"] = shadow
    d["mask_u8"] = mask
    d["free_bgr_u8"] = free
    x = to_input(shadow)
    # 480x640 native resolution: odd-size pad/crop generator (src/models/stcgan_g.py:120-132)
    g1 = stcgan_g.UnetGenerator(3, 1, ngf=64)
    g2 = stcgan_g.UnetGenerator(4, 3, ngf=64)
    g1.load_state_dict(fixture_state(g1.state_dict(), NET_SEED["G1"], "one"))
    g2.load_state_dict(fixture_state(g2.state_dict(), NET_SEED["G2"], "one"))
    g1.eval()
    g2.eval()
    with torch.no_grad():
        m_pred = g1(x)
        y_pred = g2(torch.cat((x, m_pred), dim=1))
    d["full/m_pred"] = m_pred.numpy()
    d["full/y_pred"] = y_pred.numpy()
    # train-mode forward at 480x640 (BN over padded-then-cropped positions)
    g1.train()
    g2.train()
    with torch.no_grad():
        m_t = g1(x)
        y_t = g2(torch.cat((x, m_t), dim=1))
    d["full_train/m_pred"] = m_t.numpy()
    d["full_train/y_pred"] = y_t.numpy()
    # exact 256x256 crop (no resampling) through STCGAN/networks.py
    r0, c0 = 112, 192
    xc = x[:, :, r0:r0 + 256, c0:c0 + 256].contiguous()
    n1 = networks.get_generator(3, 1, ngf=64)
    n2 = networks.get_generator(4, 3, ngf=64)
    n1.load_state_dict(fixture_state(n1.state_dict(), NET_SEED["G1"], "one"))
    n2.load_state_dict(fixture_state(n2.state_dict(), NET_SEED["G2"], "one"))
    n1.eval()
    n2.eval()
    with torch.no_grad():
        mc = n1(xc)
        yc = n2(torch.cat((xc, mc), dim=1))
    d["crop/r0c0"] = np.array([r0, c0])
    d["crop/m_pred"] = mc.numpy()
    d["crop/y_pred"] = yc.numpy()
    return d


def main():
    torch.set_num_threads(8)
    networks, loss, stcgan, stcgan_g = import_reference()
    meta = {"meta/torch": np.array(torch.__version__)}
    jobs = [
        ("nets_ngf8.npz", lambda: gen_nets(networks)),
        ("run_epoch_ngf8.npz", lambda: gen_run_epoch(networks, loss, stcgan)),
        ("g_ngf64.npz", lambda: gen_ngf64(networks)),
        ("g_ngf64_grad.npz", lambda: gen_ngf64_grad(networks, loss)),
        ("istd_114_5.npz", lambda: gen_istd(networks, stcgan_g)),
    ]
    only = set(sys.argv[1:])
    for fname, fn in jobs:
        if only and fname not in only:
            continue
        d = fn()
        d.update(meta)
        path = os.path.join(HERE, fname)
        np.savez_compressed(path, **d)
        print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB, {len(d)} entries)")


if __name__ == "__main__":
    main()
