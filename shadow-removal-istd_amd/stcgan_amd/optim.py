"""Multi-tensor Adam on one HIP launch (replaces torch.optim.Adam of STCGAN/stcgan.py:60-65).

Same constructor and ``step()/zero_grad()/state_dict()`` surface as
torch.optim.Adam for the options the reference uses (lr, betas, eps;
weight_decay=0, amsgrad=False).  The per-step pointer table is built on the
host and copied with a non-blocking H2D copy, so ``step()`` never synchronises.
"""
import torch

from . import ops
from ._lib import check, lib, ptr, stream


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False):
        if weight_decay != 0 or amsgrad:
            raise NotImplementedError("stcgan_amd Adam: weight_decay/amsgrad are not on the ST-CGAN path")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=0, amsgrad=False))
        self._epb = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self._epb is None:
            self._epb = lib().stc_adam_elems_per_block()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            # group params by step count (all equal in practice)
            by_step = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not p.is_cuda or p.dtype != torch.float32:
                    raise RuntimeError("stcgan_amd Adam: fp32 CUDA parameters only")
                if p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                    p.grad = p.grad.float().contiguous()
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                by_step.setdefault(int(st["step"].item()), []).append(p)
            for step, plist in by_step.items():
                rows, blocks = [], 0
                for p in plist:
                    st = self.state[p]
                    n = p.numel()
                    rows.append([p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                                 st["exp_avg_sq"].data_ptr(), n, blocks])
                    blocks += (n + self._epb - 1) // self._epb
                table = torch.tensor(rows, dtype=torch.int64).pin_memory().to(plist[0].device, non_blocking=True)
                check(lib().stc_adam_step(ptr(table), len(rows), blocks, float(group["lr"]), float(b1), float(b2),
                                          float(group["eps"]), int(step), stream()), "stc_adam_step")
                ops.bump(plist)
                # keep every tensor the kernel reads alive until it ran on the stream
                for p in plist:
                    p.grad.record_stream(torch.cuda.current_stream())
                table.record_stream(torch.cuda.current_stream())
        return loss
