"""Fused loss objectives (loss.d_objective / loss.g_objective, stc_loss_multi_*) vs the per-term path
(AdversarialLoss / DataLoss nodes + torch scalar arithmetic, the reference's own formulation of
STCGAN/stcgan.py:240-251, 291-299): values and every gradient bit-identical."""
import pytest
import torch

from stcgan_amd import loss

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(shape, seed, lo=-1.5, hi=1.5, grad=True):
    g = torch.Generator().manual_seed(seed)
    t = (torch.rand(shape, generator=g) * (hi - lo) + lo).to(DEV)
    return t.requires_grad_(grad)


@pytest.mark.parametrize("ls", [False, True])
@pytest.mark.parametrize("B", [1, 4, 32])
def test_d_objective_bit_identical(ls, B):
    adv = loss.AdversarialLoss(ls=ls).to(DEV)
    C = [_t((B, 1, 30, 30), s) for s in (1, 2, 3, 4)]
    C1f, C1r, C2f, C2r = C
    d1 = (adv(C1f, is_real=False) + adv(C1r, is_real=True)) * 0.5
    d2 = (adv(C2f, is_real=False) + adv(C2r, is_real=True)) * 0.5
    d = 0.1 * d1 + 0.1 * d2
    ref_g = torch.autograd.grad(d, C)
    D, D1, D2 = loss.d_objective(adv, C1f, C1r, C2f, C2r, 0.1, 0.1)
    got_g = torch.autograd.grad(D, C)
    assert torch.equal(D1, d1.detach()) and torch.equal(D2, d2.detach()) and torch.equal(D, d.detach())
    for a, b in zip(got_g, ref_g):
        assert torch.equal(a, b)


@pytest.mark.parametrize("ls", [False, True])
@pytest.mark.parametrize("B", [1, 4])
def test_g_objective_bit_identical(ls, B):
    adv = loss.AdversarialLoss(ls=ls).to(DEV)
    dl = loss.DataLoss()
    m_pred, y_pred = _t((B, 1, 64, 48), 5), _t((B, 3, 64, 48), 6)
    m, y = _t((B, 1, 64, 48), 7, grad=False), _t((B, 3, 64, 48), 8, grad=False)
    C1f, C2f = _t((B, 1, 30, 30), 9), _t((B, 1, 30, 30), 10)
    ins = [m_pred, y_pred, C1f, C2f]
    g1, g2 = adv(C1f, is_real=True), adv(C2f, is_real=True)
    a1, a2 = dl(m_pred, m), dl(y_pred, y)
    g = a1 + 5 * a2 + 0.1 * g1 + 0.1 * g2
    ref = torch.autograd.grad(g, ins)
    G, G1, G2, A1, A2 = loss.g_objective(adv, m_pred, m, y_pred, y, C1f, C2f, 5, 0.1, 0.1)
    got = torch.autograd.grad(G, ins)
    for a, b in ((G, g), (G1, g1), (G2, g2), (A1, a1), (A2, a2)):
        assert torch.equal(a.detach(), b.detach())
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


def test_objective_partial_grads():
    """Only the inputs that need a gradient get one (the D step's detached fakes)."""
    adv = loss.AdversarialLoss().to(DEV)
    C1f, C1r = _t((2, 1, 30, 30), 1, grad=False), _t((2, 1, 30, 30), 2)
    C2f, C2r = _t((2, 1, 30, 30), 3, grad=False), _t((2, 1, 30, 30), 4)
    D, _, _ = loss.d_objective(adv, C1f, C1r, C2f, C2r, 0.1, 0.1)
    D.backward()
    assert C1r.grad is not None and C2r.grad is not None
