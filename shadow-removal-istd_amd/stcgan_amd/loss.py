"""Drop-in replacement for the loss modules of STCGAN/loss.py on the ST-CGAN path.

DataLoss (STCGAN/loss.py:14-26) and AdversarialLoss (STCGAN/loss.py:59-86) run as
HIP reduction kernels (deterministic two-level sums) with hand-written gradients.
VisualLoss and SoftAdapt are not on the path.
"""
import torch
import torch.nn as nn

from . import _lib as L
from ._lib import check, lib, ptr, stream


class _LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, kind, c, pred, target):
        pred = pred.contiguous()
        if pred.dtype != torch.float32:
            raise TypeError("stcgan_amd losses take fp32 inputs")
        if not pred.is_cuda:
            raise RuntimeError("stcgan_amd losses run on the GPU only")
        if target is not None:
            target = target.contiguous()
            if target.shape != pred.shape:
                raise ValueError(f"loss: target shape {tuple(target.shape)} != prediction {tuple(pred.shape)}")
        n = pred.numel()
        part = torch.empty(max(1, lib().stc_loss_parts(n)), dtype=torch.float32, device=pred.device)
        out = torch.empty((), dtype=torch.float32, device=pred.device)
        check(lib().stc_loss_fwd(kind, ptr(pred), ptr(target), float(c), n, ptr(part), ptr(out), stream()),
              "stc_loss_fwd")
        ctx.kind, ctx.c = kind, c
        ctx.save_for_backward(pred, target if target is not None else pred)
        ctx.has_t = target is not None
        return out

    @staticmethod
    def backward(ctx, gout):
        pred, target = ctx.saved_tensors
        t = target if ctx.has_t else None
        grad = torch.empty_like(pred)
        gout = gout.contiguous().float()
        check(lib().stc_loss_bwd(ctx.kind, ptr(pred), ptr(t), float(ctx.c), pred.numel(), ptr(gout), ptr(grad),
                                 stream()), "stc_loss_bwd")
        return None, None, grad, None


def l1_loss(pred, target):
    """F.l1_loss(pred, target, reduction='mean')."""
    return _LossFn.apply(L.LOSS_L1, 0.0, pred, target)


def mse_const(pred, value):
    """F.mse_loss(pred, full_like(pred, value))."""
    return _LossFn.apply(L.LOSS_MSE_CONST, float(value), pred, None)


def bce_logits_const(pred, value):
    """F.binary_cross_entropy_with_logits(pred, full_like(pred, value))."""
    return _LossFn.apply(L.LOSS_BCE_CONST, float(value), pred, None)


class DataLoss(nn.Module):
    """Loss between shadow parameters: L1, mean reduction (STCGAN/loss.py:14-26)."""
    __slots__ = ["reduction", "norm"]

    def __init__(self, norm=None, reduction: str = 'mean'):
        super().__init__()
        if reduction != 'mean' or (norm is not None and norm is not torch.nn.functional.l1_loss):
            raise NotImplementedError("stcgan_amd DataLoss: only F.l1_loss with reduction='mean' is on the path")
        self.reduction = reduction

    def forward(self, y_pred, y_target):
        return l1_loss(y_pred, y_target)


class AdversarialLoss(nn.Module):
    """Objective of a conditional GAN (STCGAN/loss.py:59-86).

    ls=False: labels real=1 / fake=0 and F.mse_loss -- the branch the reference
    always takes (its constructor compares against the misspelt 'leastsqure',
    STCGAN/stcgan.py:111-112).  ls=True: labels 1 / -1 and BCE-with-logits,
    exactly as the reference (inverted) branches."""

    def __init__(self, ls=False, rel=False, avg=False):
        super().__init__()
        if not ls:
            self.register_buffer('real_label', torch.tensor(1.0))
            self.register_buffer('fake_label', torch.tensor(0.0))
        else:
            self.register_buffer('real_label', torch.tensor(1.0))
            self.register_buffer('fake_label', torch.tensor(-1.0))
        self.ls = ls
        self.rel = rel
        self.avg = avg
        self._labels = (1.0, -1.0 if ls else 0.0)

    def forward(self, D_out, is_real):
        target = self._labels[0] if is_real else self._labels[1]
        if not self.ls:
            return mse_const(D_out, target)
        return bce_logits_const(D_out, target)


class RelativisticAdversarialLoss(nn.Module):
    """The ``src/`` line's AdversarialLoss (src/loss.py:59-112): SGAN / RpGAN (rel) / RaGAN
    (rel + avg) objectives over a (C_real, C_fake) pair, for the discriminator (``D_loss=True``)
    or the generator; labels real=1, fake=0 (MSE) or 1 / -1 with ``ls=True`` (BCE-with-logits),
    as the reference.  The reductions and their gradients run in the HIP loss kernels; the
    relativistic differences (C_real - C_fake, C - mean over dim 0) are torch ops on the
    [B, 1, 30, 30] logits."""

    def __init__(self, ls=False, rel=False, avg=False):
        super().__init__()
        self.register_buffer('real_label', torch.tensor(1.0))
        self.register_buffer('fake_label', torch.tensor(-1.0 if ls else 0.0))
        self.ls, self.rel, self.avg = ls, rel, avg
        self._labels = (1.0, -1.0 if ls else 0.0)

    def cal_loss(self, C_out, label):
        return bce_logits_const(C_out, label) if self.ls else mse_const(C_out, label)

    def forward(self, C_real, C_fake, D_loss=True):
        real, fake = self._labels
        if self.rel and self.avg:  # RaGAN
            if D_loss:
                return (self.cal_loss(C_real - C_fake.mean(dim=0), real)
                        + self.cal_loss(C_fake - C_real.mean(dim=0), fake)) * 0.5
            return (self.cal_loss(C_real - C_fake.mean(dim=0), fake)
                    + self.cal_loss(C_fake - C_real.mean(dim=0), real)) * 0.5
        if self.rel:  # RpGAN
            return self.cal_loss(C_real - C_fake, real) if D_loss else self.cal_loss(C_fake - C_real, real)
        if D_loss:  # SGAN
            return (self.cal_loss(C_real, real) + self.cal_loss(C_fake, fake)) * 0.5
        return self.cal_loss(C_fake, real)
