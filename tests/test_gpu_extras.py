"""GPU tests of the src/ line extras: the relativistic AdversarialLoss of
src/loss.py:59-112 (values and gradients against the torch formulas of the reference, fp32,
rtol 1e-6) and the full-state checkpoint of src/cgan.py:494-523 (a resumed trainer's next
train step is bit-identical to the uninterrupted one)."""
import types

import pytest
import torch
import torch.nn.functional as F

from stcgan_amd.loss import RelativisticAdversarialLoss

pytestmark = pytest.mark.gpu


def _ref(C_real, C_fake, D_loss, ls, rel, avg):
    """src/loss.py:59-112 verbatim semantics in torch (CPU)."""
    real, fake = torch.tensor(1.0), torch.tensor(-1.0 if ls else 0.0)

    def cal(c, lab):
        return F.binary_cross_entropy_with_logits(c, lab.expand_as(c)) if ls else F.mse_loss(c, lab.expand_as(c))
    if D_loss:
        if rel and avg:
            return (cal(C_real - C_fake.mean(dim=0), real) + cal(C_fake - C_real.mean(dim=0), fake)) * 0.5
        if rel:
            return cal(C_real - C_fake, real)
        return (cal(C_real, real) + cal(C_fake, fake)) * 0.5
    if rel and avg:
        return (cal(C_real - C_fake.mean(dim=0), fake) + cal(C_fake - C_real.mean(dim=0), real)) * 0.5
    if rel:
        return cal(C_fake - C_real, real)
    return cal(C_fake, real)


@pytest.mark.parametrize("ls", [False, True])
@pytest.mark.parametrize("rel,avg", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("D_loss", [True, False])
def test_relativistic_loss_matches_reference(ls, rel, avg, D_loss):
    g = torch.Generator().manual_seed(int(ls) * 8 + int(rel) * 4 + int(avg) * 2 + int(D_loss))
    cr, cf = torch.randn((4, 1, 30, 30), generator=g), torch.randn((4, 1, 30, 30), generator=g)
    a, b = cr.clone().requires_grad_(), cf.clone().requires_grad_()
    want = _ref(a, b, D_loss, ls, rel, avg)
    want.backward()
    x, y = cr.cuda().requires_grad_(), cf.cuda().requires_grad_()
    got = RelativisticAdversarialLoss(ls, rel, avg).cuda()(x, y, D_loss=D_loss)
    got.backward()
    assert abs(float(got) - float(want)) <= 1e-6 * max(1.0, abs(float(want)))
    for got_g, ref_g in ((x.grad, a.grad), (y.grad, b.grad)):
        assert (got_g is None) == (ref_g is None)  # the SGAN generator loss ignores C_real
        if ref_g is not None:
            torch.testing.assert_close(got_g.cpu(), ref_g, rtol=1e-5, atol=1e-9)


def _trainer(seed):
    from stcgan_amd.stcgan import STCGAN
    torch.manual_seed(seed)
    a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                              D_loss_fn="standard", D_loss_type="normal", ngf=8, dtype="fp32",
                              load_weights_g1=None, load_weights_g2=None, load_weights_d1=None,
                              load_weights_d2=None)
    return STCGAN(a)


def test_checkpoint_resume_is_bit_identical(tmp_path):
    g = torch.Generator().manual_seed(0)
    batches = [tuple(torch.rand((2, c, 256, 256), generator=g).cuda() * 2 - 1 for c in (3, 1, 3)) for _ in range(2)]
    t1 = _trainer(1)
    t1.train_step(*batches[0])
    path = str(tmp_path / "checkpoint.tar")
    t1.save_checkpoint(7, path)
    t2 = _trainer(2)  # different initial weights
    t2.load_checkpoint(path)
    assert t2.start_epoch == 7
    l1 = t1.train_step(*batches[1])
    l2 = t2.train_step(*batches[1])
    for k in l1:
        assert float(l1[k]) == float(l2[k]), k
    for n in ("G1", "G2", "D1", "D2"):
        s1, s2 = getattr(t1, n).state_dict(), getattr(t2, n).state_dict()
        for k in s1:
            assert torch.equal(s1[k], s2[k]), (n, k)


@pytest.mark.parametrize("dtype,loss_type", [("bf16", "normal"), ("fp32", "rel_avg")])
def test_side_stream_step_is_bit_identical(dtype, loss_type):
    """Discriminators on side HIP streams (STCGAN.streams) vs the one-stream step: same kernels in
    the same per-network order, so three steps leave bit-identical states and losses."""
    from stcgan_amd.stcgan import STCGAN
    g = torch.Generator().manual_seed(3)
    batches = [tuple(torch.rand((4, c, 256, 256), generator=g).cuda() * 2 - 1 for c in (3, 1, 3)) for _ in range(3)]
    out = []
    for lanes in (False, True):
        torch.manual_seed(11)
        a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                                  D_loss_fn="standard", D_loss_type=loss_type, ngf=64, dtype=dtype, streams=lanes,
                                  load_weights_g1=None, load_weights_g2=None, load_weights_d1=None,
                                  load_weights_d2=None)
        tr = STCGAN(a)
        losses = [tr.train_step(*b) for b in batches]
        torch.cuda.synchronize()
        out.append((losses, {n: getattr(tr, n).state_dict() for n in ("G1", "G2", "D1", "D2")}))
    (l0, s0), (l1, s1) = out
    for a_, b_ in zip(l0, l1):
        for k in a_:
            assert float(a_[k]) == float(b_[k]), k
    for n in s0:
        for k in s0[n]:
            assert torch.equal(s0[n][k], s1[n][k]), (n, k)
