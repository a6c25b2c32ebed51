"""Multi-tensor Adam on one HIP launch (replaces torch.optim.Adam of STCGAN/stcgan.py:60-65).

Same constructor and ``step()/zero_grad()/state_dict()`` surface as
torch.optim.Adam for the options the reference uses (lr, betas, eps;
weight_decay=0, amsgrad=False).  The pointer table lives on the device and is
rebuilt only when a tensor moved; ``step()`` never synchronises.  The 4x4
weights' packed GEMM operands (ops.packed) are rewritten in the same launch as
the update (stc_adam_pack_step), so the next forward finds them fresh.
"""
import torch

from . import _lib as L

from . import ops
from ._lib import check, lib, ptr, stream


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False):
        if weight_decay != 0 or amsgrad:
            raise NotImplementedError("stcgan_amd Adam: weight_decay/amsgrad are not on the ST-CGAN path")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=0, amsgrad=False))
        self._epb = None
        self.fuse_pack = True  # False: update only (the packed operands are then refreshed lazily)

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
            self._fast = {}     # group -> the last step's table and per-parameter records (see _fast_step)
        for gi, group in enumerate(self.param_groups):
            if self._fast_step(gi, group):
                continue
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
                recs = [self._record(p) for p in plist]
                key = tuple(r[0] for r in recs)
                cached = self._tables.get(gi)
                if cached is not None and cached[0] == key:
                    table, blocks = cached[1], cached[2]
                else:
                    # pointer table, rebuilt when a tensor or packed operand moved (the gradients are new
                    # tensors every step, so in practice every step: a few hundred rows)
                    rows, blocks = [], 0
                    for row, nblk, _ in recs:
                        rows.append(list(row[:5]) + [blocks] + list(row[5:]))
                        blocks += nblk
                    # pinned + non_blocking: a stream-ordered copy -- a pageable H2D copy would block the
                    # host until the GPU has drained everything queued before it (one full step)
                    table = torch.tensor(rows, dtype=torch.int64).pin_memory().to(plist[0].device, non_blocking=True)
                    self._tables[gi] = (key, table, blocks)
                check(lib().stc_adam_pack_step(ptr(table), len(key), blocks, float(group["lr"]), float(b1),
                                               float(b2), float(group["eps"]), int(step), stream()),
                      "stc_adam_pack_step")
                ops.bump(plist)
                for p, (_, _, targets) in zip(plist, recs):  # the packed operands written above are current
                    ver = ops.pack_version(p)
                    for (pkey, cache, out) in targets:
                        cache[pkey] = (ver, out)
            self._fast.pop(gi, None)
            if len(by_step) == 1:
                (step, plist), = by_step.items()
                recs = [self._record(p) for p in plist]
                self._fast[gi] = dict(
                    key=tuple((id(p), p.data_ptr(), p.grad.data_ptr()) for p in plist), plist=plist,
                    rows=[list(r[0]) for r in recs], table=self._tables[gi][1], blocks=self._tables[gi][2],
                    targets=[r[2] for r in recs], step=step, epoch=ops.PACK_EPOCH,
                    step_tensors=[self.state[p]["step"] for p in plist])
                f = self._fast[gi]
                f["tables"] = {f["key"]: (f["table"], f["blocks"])}
        return loss

    def _fast_step(self, gi, group):
        """The steady-state step of a group without per-parameter record building: valid while the
        parameters with a gradient, their storage, the optimiser state and every packed operand
        buffer (ops.PACK_EPOCH) are those of the previous step; only the gradients' addresses are
        read (usually unchanged: the table is then reused as is).  Returns False to take the full path."""
        f = self._fast.get(gi)
        if f is None or f["epoch"] != ops.PACK_EPOCH:
            return False
        plist = f["plist"]
        key = []
        for p in group["params"]:
            g = p.grad
            if g is None:
                continue
            if g.dtype is not torch.float32 or not g.is_contiguous():
                return False
            key.append((id(p), p.data_ptr(), g.data_ptr()))
        key = tuple(key)
        if key != f["key"]:
            if len(key) != len(f["key"]) or any(a[:2] != b[:2] for a, b in zip(key, f["key"])):
                return False
            # same parameters, other gradient buffers (the caching allocator cycles through a few address
            # patterns): a table per pattern, built once -- patch the grad column and upload
            hit = f["tables"].get(key)
            if hit is None:
                rows, blocks = [], 0
                for r, k in zip(f["rows"], key):
                    r[1] = k[2]
                for r, p in zip(f["rows"], plist):
                    rows.append(r[:5] + [blocks] + r[5:])
                    blocks += self._nblocks(p, r)
                table = torch.tensor(rows, dtype=torch.int64).pin_memory().to(plist[0].device, non_blocking=True)
                if len(f["tables"]) >= 8:
                    f["tables"].pop(next(iter(f["tables"])))
                hit = f["tables"][key] = (table, blocks)
            f["table"], f["blocks"] = hit
            f["key"] = key
            self._tables[gi] = (None, f["table"], f["blocks"])
        step = f["step"] + 1
        b1, b2 = group["betas"]
        torch._foreach_add_(f["step_tensors"], 1.0)
        check(lib().stc_adam_pack_step(ptr(f["table"]), len(plist), f["blocks"], float(group["lr"]), float(b1),
                                       float(b2), float(group["eps"]), step, stream()), "stc_adam_pack_step")
        ops.bump(plist)
        for p, targets, st in zip(plist, f["targets"], f["step_tensors"]):
            self._steps[id(p)] = (st, step)
            if targets:
                ver = ops.pack_version(p)
                for (pkey, cache, out) in targets:
                    cache[pkey] = (ver, out)
        f["step"] = step
        return True

    @staticmethod
    def _nblocks(p, row):
        if row[5]:  # packed 4x4 weight: 16x16 (p, q) tiles
            return ((p.shape[0] + 15) // 16) * row[8]
        return (p.numel() + 1023) // 1024

    def load_state_dict(self, state_dict):
        self._fast = {}
        self._steps = {}
        return super().load_state_dict(state_dict)

    def _record(self, p):
        """(table row without first_block, blocks, packed targets) of one parameter."""
        st = self.state[p]
        head = (p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), p.numel())
        is_w = self.fuse_pack and p.dim() == 4 and tuple(p.shape[2:]) == (4, 4)
        targets = ops.pack_targets(p)[:2] if is_w else []
        if not targets:
            return head + (0, 0, 0, 0, 0) + (0,) * 13, (p.numel() + 1023) // 1024, []
        P, Q = p.shape[0], p.shape[1]
        qt = (Q + 15) // 16
        packs = ()
        for (_, _, mode, out, n_pad, c_pad, dt) in targets:
            packs += (mode, out.data_ptr(), n_pad, c_pad, L.dtype_code(dt))
        packs += (0,) * (10 - len(packs))
        return (head + (1, P, Q, qt, len(targets)) + packs + (0,) * 3, ((P + 15) // 16) * qt,
                [(t[0], t[1], t[3]) for t in targets])
