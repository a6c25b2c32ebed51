"""Drop-in replacement for the loss modules of STCGAN/loss.py on the ST-CGAN path.

DataLoss (STCGAN/loss.py:14-26) and AdversarialLoss (STCGAN/loss.py:59-86) run as
HIP reduction kernels (deterministic two-level sums) with hand-written gradients.
VisualLoss and SoftAdapt are not on the path.
"""
import ctypes

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


def _arr(ctype, vals):
    return (ctype * len(vals))(*vals)


class _ObjectiveFn(torch.autograd.Function):
    """Four loss terms and the scalar arithmetic combining them as one node: two launches forward, one
    backward (stc_loss_multi_*), instead of 4 loss nodes and ~6 torch scalar ops with their own launches
    and autograd nodes.  Values bit-identical to the per-term path (same reductions, same fp32 rounding
    order).  forward -> (objective, parts): parts = the named sub-losses, not differentiable."""

    @staticmethod
    def forward(ctx, mode, kinds, consts, w, wab, *tensors):
        preds = [t.contiguous() for t in tensors[:4]]
        targets = [t.contiguous() if t is not None else None for t in tensors[4:]]
        for p_, t_ in zip(preds, targets):
            if p_.dtype != torch.float32 or not p_.is_cuda:
                raise TypeError("stcgan_amd losses take fp32 CUDA inputs")
            if t_ is not None and t_.shape != p_.shape:
                raise ValueError(f"loss: target shape {tuple(t_.shape)} != prediction {tuple(p_.shape)}")
        dev = preds[0].device
        numels = [p_.numel() for p_ in preds]
        l = lib()
        n_arr = _arr(ctypes.c_int64, numels)
        part = torch.empty(l.stc_loss_multi_parts(4, n_arr), dtype=torch.float32, device=dev)
        vals = torch.empty(6, dtype=torch.float32, device=dev)  # the 4 terms, then D1, D2 (mode D)
        total = torch.empty((), dtype=torch.float32, device=dev)
        args = (4, _arr(ctypes.c_int32, kinds), _arr(ctypes.c_float, consts),
                _arr(ctypes.c_void_p, [p_.data_ptr() for p_ in preds]),
                _arr(ctypes.c_void_p, [t_.data_ptr() if t_ is not None else None for t_ in targets]), n_arr)
        check(l.stc_loss_multi_fwd(*args, mode, _arr(ctypes.c_float, list(w) + [0.0] * (3 - len(w))), ptr(part),
                                   ptr(vals), ptr(total), stream()), "stc_loss_multi_fwd")
        ctx.args, ctx.wab = args, wab
        ctx.save_for_backward(*preds, *[t_ if t_ is not None else preds[0] for t_ in targets])
        ctx.mark_non_differentiable(vals)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the non-differentiable parts
        return total, vals

    @staticmethod
    def backward(ctx, gout, _gparts):
        if gout is None:
            return (None,) * 13
        preds = ctx.saved_tensors[:4]
        need = ctx.needs_input_grad[5:9]
        grads = [torch.empty_like(p_) if nd else None for p_, nd in zip(preds, need)]
        wa, wb = ctx.wab
        gout = gout.contiguous().float()
        check(lib().stc_loss_multi_bwd(*ctx.args, _arr(ctypes.c_float, wa), _arr(ctypes.c_float, wb), ptr(gout),
                                       _arr(ctypes.c_void_p, [g.data_ptr() if g is not None else None
                                                              for g in grads]), stream()), "stc_loss_multi_bwd")
        return (None,) * 5 + tuple(grads) + (None,) * 4


def d_objective(adv, C1_fake, C1_real, C2_fake, C2_real, lambda2, lambda3):
    """The D objective of STCGAN/stcgan.py:240-251 (loss type "normal"):
    D1 = (adv(C1_fake, fake) + adv(C1_real, real)) * 0.5, D2 likewise, D = lambda2*D1 + lambda3*D2.
    Returns (D, D1, D2)."""
    real, fake = adv._labels
    k = L.LOSS_BCE_CONST if adv.ls else L.LOSS_MSE_CONST
    total, parts = _ObjectiveFn.apply(L.LOSS_COMBINE_D, [k] * 4, [fake, real, fake, real], [lambda2, lambda3],
                                      ([lambda2, lambda2, lambda3, lambda3], [0.5] * 4),
                                      C1_fake, C1_real, C2_fake, C2_real, None, None, None, None)
    return total, parts[4], parts[5]


def d_term_grad(adv, C, lam, gout, real=True):
    """d_objective's gradient with respect to one of its four logits tensors, lam * 0.5 * adv'(C, label) (label: real
    or fake) scaled by the objective's incoming gradient ``gout`` (fp32 device scalar) -- the same per-term kernel
    arithmetic as that node's backward (stc_loss_multi_bwd), available as soon as C is: with loss type normal each
    term involves one logits tensor only, so each discriminator call's backward need not wait for the other calls
    (STCGAN.train_step runs them early; the objective then takes the logits detached)."""
    label = adv._labels[0] if real else adv._labels[1]
    k = L.LOSS_BCE_CONST if adv.ls else L.LOSS_MSE_CONST
    p_ = C.contiguous()
    if p_.dtype != torch.float32 or not p_.is_cuda:
        raise TypeError("stcgan_amd losses take fp32 CUDA inputs")
    g = torch.empty_like(p_)
    check(lib().stc_loss_multi_bwd(1, _arr(ctypes.c_int32, [k]), _arr(ctypes.c_float, [label]),
                                   _arr(ctypes.c_void_p, [p_.data_ptr()]), _arr(ctypes.c_void_p, [None]),
                                   _arr(ctypes.c_int64, [p_.numel()]), _arr(ctypes.c_float, [lam]),
                                   _arr(ctypes.c_float, [0.5]), ptr(gout), _arr(ctypes.c_void_p, [g.data_ptr()]),
                                   stream()), "stc_loss_multi_bwd")
    return g


def g_objective(adv, m_pred, m, y_pred, y, C1_fake, C2_fake, lambda1, lambda2, lambda3):
    """The G objective of STCGAN/stcgan.py:291-299 (loss type "normal"): G1 = adv(C1_fake, real),
    G2 = adv(C2_fake, real), data1 = L1(m_pred, m), data2 = L1(y_pred, y),
    G = data1 + lambda1*data2 + lambda2*G1 + lambda3*G2.  Returns (G, G1, G2, data1, data2)."""
    real = adv._labels[0]
    k = L.LOSS_BCE_CONST if adv.ls else L.LOSS_MSE_CONST
    total, v = _ObjectiveFn.apply(L.LOSS_COMBINE_G, [L.LOSS_L1, L.LOSS_L1, k, k], [0.0, 0.0, real, real],
                                  [lambda1, lambda2, lambda3], ([1.0, lambda1, lambda2, lambda3], [1.0] * 4),
                                  m_pred, y_pred, C1_fake, C2_fake, m, y, None, None)
    return total, v[2], v[3], v[0], v[1]


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
