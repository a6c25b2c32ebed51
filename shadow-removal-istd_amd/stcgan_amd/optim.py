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
        self._dev = None  # device-resident step counts (device_step), per group
        self._ov_stream = None  # overlap(): the side stream of the per-bucket updates
        self._ov_done = {}      # group -> {position in the group's steady-state plist} updated this step
        self._ov_coef = set()   # groups whose device step count this step already advanced
        self._gi_of = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._init_state()
        for gi, group in enumerate(self.param_groups):
            done = self._ov_done.pop(gi, None)
            if done:
                self._finish_overlap(gi, group, done)
                continue
            if self._fast_step(gi, group):
                continue
            self._full_step(gi, group)
        self._ov_coef.clear()
        return loss

    def _init_state(self):
        if self._epb is None:
            self._epb = lib().stc_adam_elems_per_block()
            self._steps = {}    # id(param) -> (state step tensor, its value as a Python int)
            self._tables = {}   # (group, step) -> (pointer key, device table, blocks)
            self._fast = {}     # group -> the last step's table and per-parameter records (see _fast_step)

    def _full_step(self, gi, group, skip=()):
        """The general path (first steps, moved tensors, new packed operands); ``skip``: parameters already
        updated this step (by overlap), left out.  With device-resident step counts (device_step) the host
        counts are first brought level with the device counter (replays advance only that), and the counter
        is set to the count this step reaches, so the next steady-state step (or replay) continues from it."""
        if self._dev is not None and gi in self._dev:
            self._pull_device_steps(gi, skip)
        b1, b2 = group["betas"]
        # group params by step count (all equal in practice).  The step count is mirrored in a
        # Python int (no per-parameter tensor op / .item() on the host path), and the state's
        # "step" tensors are advanced with one foreach call.
        by_step, step_tensors = {}, []
        for p in group["params"]:
            if p.grad is None or id(p) in skip:
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
        if self._dev is not None and gi in self._dev and len(by_step) == 1:
            (step,), = (tuple(by_step),)
            self._dev[gi]["step"].fill_(int(step))  # (stream-ordered; a captured graph keeps this tensor)
        self._fast.pop(gi, None)
        if len(by_step) == 1 and not skip:
            (step, plist), = by_step.items()
            recs = [self._record(p) for p in plist]
            self._fast[gi] = dict(
                key=tuple((id(p), p.data_ptr(), p.grad.data_ptr()) for p in plist), plist=plist,
                rows=[list(r[0]) for r in recs], table=self._tables[gi][1], blocks=self._tables[gi][2],
                targets=[r[2] for r in recs], step=step, epoch=ops.PACK_EPOCH,
                step_tensors=[self.state[p]["step"] for p in plist],
                index={id(p): i for i, p in enumerate(plist)}, subs={})
            f = self._fast[gi]
            f["tables"] = {f["key"]: (f["table"], f["blocks"])}

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
            f["subs"] = {}  # subset tables hold the old gradient addresses
            self._tables[gi] = (None, f["table"], f["blocks"])
        step = f["step"] + 1
        b1, b2 = group["betas"]
        torch._foreach_add_(f["step_tensors"], 1.0)
        if self._dev is not None:
            d = self._dev_state(gi, group, f["step"], plist[0].device)
            check(lib().stc_adam_pack_step_dev(ptr(f["table"]), len(plist), f["blocks"], ptr(d["step"]), ptr(d["lr_dev"]),
                                               ptr(d["bc1"]), ptr(d["bc2s"]), d["tab_len"], ptr(d["coef"]), float(b1),
                                               float(b2), float(group["eps"]), stream()), "stc_adam_pack_step_dev")
        else:
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

    # ------------------------------------------------------------------ overlap with the backward
    def overlap(self, exchanges, on=True):
        """Update the parameters bucket by bucket while the backward still runs.  Each network's gradient
        buckets (parallel.BucketExchange, fed by engine.GradWriter) are handed over the moment the backward
        has written them and no longer reads their parameters (a layer is reported after its input-gradient
        convolution); the bucket's update is launched on a side stream ordered after the streams that wrote
        it and after its all-reduce.  ``step()`` updates what is left and joins the side stream.  Every
        tensor's update is the same kernel arithmetic on the same values as one whole-group launch (Adam
        updates each tensor independently), so results are bit-identical; only the steady state overlaps (a
        first step, a moved tensor or a new packed operand leaves everything to step())."""
        for ex in exchanges:
            ex.on_complete = self._bucket_ready if on else None

    def _bucket_ready(self, params, stream, work):
        if self._epb is None:
            return
        if self._gi_of is None:
            self._gi_of = {id(p): gi for gi, g in enumerate(self.param_groups) for p in g["params"]}
        by_group = {}
        for p in params:
            gi = self._gi_of.get(id(p))
            if gi is not None:
                by_group.setdefault(gi, []).append(p)
        for gi, ps in by_group.items():
            self._launch_subset(gi, ps, stream, work)

    def _subset(self, f, sel):
        """(device table, blocks) of the steady-state records at positions ``sel`` (cached)."""
        key = tuple(sel)
        sub = f["subs"].get(key)
        if sub is None:
            rows, blocks = [], 0
            for i in sel:
                r = f["rows"][i]
                rows.append(r[:5] + [blocks] + r[5:])
                blocks += self._nblocks(f["plist"][i], r)
            dev = f["plist"][0].device
            sub = f["subs"][key] = (torch.tensor(rows, dtype=torch.int64).pin_memory().to(dev, non_blocking=True),
                                    blocks)
        return sub

    def _launch_subset(self, gi, ps, stream, work):
        f = self._fast.get(gi)
        if f is None or f["epoch"] != ops.PACK_EPOCH:
            return
        done = self._ov_done.get(gi, {})
        sel = []
        for p in ps:
            i = f["index"].get(id(p))
            g = p.grad
            if (i is None or i in done or g is None or g.dtype is not torch.float32 or not g.is_contiguous()
                    or g.data_ptr() != f["rows"][i][1] or p.data_ptr() != f["rows"][i][0]):
                return  # left to step()
            sel.append(i)
        sel.sort()
        if tuple(sel) not in f["subs"] and torch.cuda.is_current_stream_capturing():
            return  # (no table upload inside a capture)
        table, blocks = self._subset(f, sel)
        dev = f["plist"][0].device
        if self._ov_stream is None:
            self._ov_stream = torch.cuda.Stream(dev)
        ost = self._ov_stream
        ost.wait_stream(torch.cuda.current_stream(dev))
        if stream is not None:
            ost.wait_stream(stream)
        with torch.cuda.stream(ost):
            if work is not None:
                work.wait()
            self._apply(gi, f, table, len(sel), blocks)
        self._ov_done.setdefault(gi, {}).update((i, True) for i in sel)

    def _apply(self, gi, f, table, n, blocks):
        """One table launch of this step's update of group ``gi`` on the current stream."""
        group = self.param_groups[gi]
        b1, b2 = group["betas"]
        coef = None
        if self._dev is not None:
            d = self._dev_state(gi, group, f["step"], f["plist"][0].device)
            if gi not in self._ov_coef:  # the device step count advances once per step
                check(lib().stc_adam_coef_dev(ptr(d["step"]), ptr(d["lr_dev"]), ptr(d["bc1"]), ptr(d["bc2s"]),
                                              d["tab_len"], ptr(d["coef"]), stream()), "stc_adam_coef_dev")
                self._ov_coef.add(gi)
            coef = ptr(d["coef"])
        check(lib().stc_adam_pack_apply(ptr(table), n, blocks, float(group["lr"]), f["step"] + 1, coef, float(b1),
                                        float(b2), float(group["eps"]), stream()), "stc_adam_pack_apply")

    def _finish_overlap(self, gi, group, done):
        """step() of a group part of which overlap() already updated this step."""
        f = self._fast[gi]
        plist = f["plist"]
        torch.cuda.current_stream(plist[0].device).wait_stream(self._ov_stream)
        with_grad = [p for p in group["params"] if p.grad is not None]
        ok = f["epoch"] == ops.PACK_EPOCH and len(with_grad) == len(plist)
        rest = []
        for p in with_grad:
            i = f["index"].get(id(p))
            if i is None:
                ok = False
                break
            if i in done:
                continue
            g = p.grad
            if (g.dtype is not torch.float32 or not g.is_contiguous() or g.data_ptr() != f["rows"][i][1]
                    or p.data_ptr() != f["rows"][i][0]):
                ok = False
            rest.append(i)
        step = f["step"] + 1
        if ok:
            if rest:
                table, blocks = self._subset(f, rest)
                self._apply(gi, f, table, len(rest), blocks)
            torch._foreach_add_(f["step_tensors"], 1.0)
            upd = plist
        else:  # the rest on the general path; the updated part's host-side state advanced here
            upd = [plist[i] for i in done]
            if self._dev is not None and gi in self._dev:
                self._pull_device_steps(gi, {id(p) for p in upd})  # (device counts: already advanced)
                step = f["step"] + 1
            else:
                torch._foreach_add_([f["step_tensors"][i] for i in done], 1.0)
        ops.bump(upd)
        for p in upd:
            i = f["index"][id(p)]
            self._steps[id(p)] = (f["step_tensors"][i], step)
            ver = ops.pack_version(p)
            for (pkey, cache, out) in f["targets"][i]:
                cache[pkey] = (ver, out)
        if ok:
            f["step"] = step
        else:
            self._full_step(gi, group, skip={id(p) for p in upd})

    def zero_grad(self, set_to_none=True):
        if self._ov_done:  # a backward overlapped some updates and no step() followed: finish them
            self.step()
        super().zero_grad(set_to_none=set_to_none)

    # ------------------------------------------------------------------ device-resident step count
    def device_step(self, on=True, tab_len=1 << 17):
        """Keep each parameter group's step count on the device (stc_adam_pack_step_dev), so that a train
        step captured as a HIP graph advances it at every replay; the host-side counts are brought back by
        sync_steps() (state_dict() does it).  The steady-state path only: call after one ordinary step."""
        if on and self._dev is None:
            self._dev = {}
            self._tab_len = int(tab_len)
        elif not on and self._dev is not None:
            self.sync_steps()
            self._dev = None

    def _dev_state(self, gi, group, host_step, device):
        import math
        import numpy as np
        d = self._dev.get(gi)
        if d is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("stcgan_amd Adam: the device step state is made by an eager step, not in a capture")
            b1, b2 = (float(np.float32(b)) for b in group["betas"])  # the float betas the kernel receives
            n = self._tab_len
            # exactly the host path's formulas: 1 - pow(beta1, step) in double; (float)sqrt(1 - pow(beta2, step))
            bc1 = [1.0] + [1.0 - math.pow(b1, float(k)) for k in range(1, n)]
            bc2s = [1.0] + [math.sqrt(1.0 - math.pow(b2, float(k))) for k in range(1, n)]
            d = dict(tab_len=n, lr=None,
                     bc1=torch.tensor(bc1, dtype=torch.float64, device=device),
                     bc2s=torch.tensor(np.asarray(bc2s, dtype=np.float64).astype(np.float32), device=device),
                     step=torch.tensor([int(host_step)], dtype=torch.int64, device=device),
                     lr_dev=torch.zeros(1, dtype=torch.float64, device=device),
                     coef=torch.zeros(2, dtype=torch.float32, device=device))
            self._dev[gi] = d
        if host_step + 1 >= d["tab_len"]:
            raise RuntimeError("stcgan_amd Adam: device step table exhausted; device_step(tab_len=...) larger")
        if d["lr"] != group["lr"]:  # the double value of the float lr the host path passes
            d["lr_dev"].fill_(float(np.float32(group["lr"])))
            d["lr"] = group["lr"]
        return d

    def sync_lr(self):
        """Push a changed learning rate (a scheduler step) to the device copies the captured step reads."""
        if not self._dev:
            return
        import numpy as np
        for gi, d in self._dev.items():
            lr = self.param_groups[gi]["lr"]
            if d["lr"] != lr:
                d["lr_dev"].fill_(float(np.float32(lr)))
                d["lr"] = lr

    def _pull_device_steps(self, gi, updated=()):
        """Host step counts of group ``gi`` from its device counter: parameters whose update of this step already
        ran (``updated``: ids) get the count this step reaches, the others the count before it."""
        d, f = self._dev.get(gi), self._fast.get(gi)
        if d is None:
            return
        s = int(d["step"].item())
        if f is None:  # (no steady-state record, e.g. after load_state_dict -- which set the counter -- and replays)
            for p in self.param_groups[gi]["params"]:
                st = self.state.get(p)
                if st and "step" in st:
                    st["step"].fill_(float(s))
                    self._steps.pop(id(p), None)
            return
        if gi in self._ov_coef:  # this step's advance already happened (overlapped bucket updates)
            s -= 1
        for p, st in zip(f["plist"], f["step_tensors"]):
            v = s + 1 if id(p) in updated else s
            st.fill_(float(v))
            self._steps[id(p)] = (st, v)
        f["step"] = s

    def sync_steps(self):
        """Host step counts (state["step"], the steady-state mirrors) from the device counters."""
        if not self._dev:
            return
        for gi, d in self._dev.items():
            s = int(d["step"].item())
            f = self._fast.get(gi)
            if f is None:  # (no steady-state record -- e.g. replays after load_state_dict: every state of the group)
                for p in self.param_groups[gi]["params"]:
                    st = self.state.get(p)
                    if st and "step" in st:
                        st["step"].fill_(float(s))
                        self._steps.pop(id(p), None)
                continue
            f["step"] = s
            for p, st in zip(f["plist"], f["step_tensors"]):
                st.fill_(float(s))
                self._steps[id(p)] = (st, s)

    def state_dict(self):
        self.sync_steps()
        return super().state_dict()

    @staticmethod
    def _nblocks(p, row):
        if row[5]:  # packed 4x4 weight: 16x16 (p, q) tiles
            return ((p.shape[0] + 15) // 16) * row[8]
        return (p.numel() + 1023) // 1024

    def load_state_dict(self, state_dict):
        if self._ov_done:  # updates of an overlapped backward that no step() finished
            self.step()
        self._fast = {}
        self._steps = {}
        self._ov_done = {}
        # the moment buffers keep their storage: a captured graph (STCGAN.capture) and its pointer tables hold
        # their addresses, so the loaded values are copied into them rather than swapped in as new tensors
        held = {id(p): (p, {k: v for k, v in self.state[p].items() if k in ("exp_avg", "exp_avg_sq")})
                for g in self.param_groups for p in g["params"] if p in self.state}
        out = super().load_state_dict(state_dict)
        for p, old in held.values():
            st = self.state.get(p)
            if st is None:
                continue
            for k, t in old.items():
                new = st.get(k)
                if new is not None and new is not t and new.shape == t.shape:
                    t.copy_(new)
                    st[k] = t
        # device-resident counts (device_step): the loaded state's; the counter tensors are kept (a captured
        # graph holds them), the next step takes the general path and writes them
        if self._dev:
            for gi, d in self._dev.items():
                st = [self.state[p]["step"] for p in self.param_groups[gi]["params"] if "step" in self.state[p]]
                if st:
                    d["step"].fill_(int(st[0].item()))
        return out

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
