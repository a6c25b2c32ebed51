"""Multi-tensor Adam on one HIP launch (replaces torch.optim.Adam of STCGAN/stcgan.py:60-65).

Same constructor and ``step()/zero_grad()/state_dict()`` surface as
torch.optim.Adam for the options the reference uses (lr, betas, eps;
weight_decay=0, amsgrad=False).  The pointer table lives on the device and is
rebuilt only when a tensor moved; ``step()`` never synchronises.
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
            self._steps = {}    # id(param) -> (state step tensor, its value as a Python int)
            self._tables = {}   # (group, step) -> (pointer key, device table, blocks)
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            # group params by step count (all equal in practice).  The step count is mirrored in a
            # Python int (no per-parameter tensor op / .item() on the host path), and the state's
            # "step" tensors are advanced with one foreach call.
            by_step, step_tensors = {}, []
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
                mirror = self._steps.get(id(p))
                n = mirror[1] + 1 if mirror is not None and mirror[0] is st["step"] else int(st["step"].item()) + 1
                self._steps[id(p)] = (st["step"], n)
                step_tensors.append(st["step"])
                by_step.setdefault(n, []).append(p)
            if step_tensors:
                torch._foreach_add_(step_tensors, 1.0)
            for step, plist in by_step.items():
                key = tuple((p.data_ptr(), p.grad.data_ptr(), self.state[p]["exp_avg"].data_ptr(),
                             self.state[p]["exp_avg_sq"].data_ptr(), p.numel()) for p in plist)
                cached = self._tables.get(gi)
                if cached is not None and cached[0] == key:
                    table, blocks = cached[1], cached[2]
                else:
                    # pointer table, rebuilt only when a tensor moved (the caching allocator hands the
                    # gradients the same blocks step after step); the device copy is stream-ordered
                    rows, blocks = [], 0
                    for (pp, gp, mp, vp, n) in key:
                        rows.append([pp, gp, mp, vp, n, blocks])
                        blocks += (n + self._epb - 1) // self._epb
                    table = torch.tensor(rows, dtype=torch.int64).to(plist[0].device)
                    self._tables[gi] = (key, table, blocks)
                check(lib().stc_adam_step(ptr(table), len(key), blocks, float(group["lr"]), float(b1), float(b2),
                                          float(group["eps"]), int(step), stream()), "stc_adam_step")
                ops.bump(plist)
        return loss
