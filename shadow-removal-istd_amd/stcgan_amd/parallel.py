"""Data parallelism for the ST-CGAN step: one process per GPU, RCCL over xGMI.

Replaces ``nn.DataParallel`` (STCGAN/stcgan.py:53-59).  Semantics kept from the
reference: BatchNorm statistics are per shard (each rank normalises its own
slice), the loss is the mean over the global batch (= the average of the
per-rank means for equal shards), and the running statistics that matter are
rank 0's (DataParallel keeps dev0's replica).  Exchange per optimiser step:
one all-reduce of the gradients per network (sum, then scaled by 1/world).

Overlap: every network's gradients arrive in one autograd node (engine.NetFn),
so a post-accumulate-grad hook counts arrivals per network and launches that
network's bucketed all-reduce asynchronously the moment its last gradient lands
-- G2's 218 MB exchange runs while G1's backward still computes.  ``__call__``
launches whatever did not fire, waits, and scatters the averages back.
"""
import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 1


def rank():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank()
    return 0


class GradAllReduce:
    """Average the .grad of parameter groups over all ranks.

    groups: list of parameter lists (one per network); expected[g]: how many
    backward passes accumulate into group g before one exchange (autograd sums
    the uses of a parameter inside one graph before it accumulates, so a
    network called twice in one differentiated graph still counts once).
    Each group is exchanged in flat fp32 buckets of ~bucket_mb (few, large
    collectives: ring bandwidth on xGMI is per link)."""

    def __init__(self, groups, expected=None, bucket_mb=64):
        self.groups = [[p for p in g] for g in groups]
        self.expected = list(expected) if expected is not None else [1] * len(self.groups)
        self.bucket_elems = max(1, int(bucket_mb * (1 << 20) // 4))
        self.buckets = []  # per group: list of param lists
        for g in self.groups:
            bks, cur, n = [], [], 0
            for p in g:
                cur.append(p)
                n += p.numel()
                if n >= self.bucket_elems:
                    bks.append(cur)
                    cur, n = [], 0
            if cur:
                bks.append(cur)
            self.buckets.append(bks)
        self.flat = None
        self.works = [None] * len(self.groups)
        self.count = [0] * len(self.groups)
        self.hooks = []
        self.overlap = False

    # ---- hooks --------------------------------------------------------------------
    def enable_overlap(self):
        """Launch each group's exchange from the backward as soon as it is complete."""
        if self.overlap or world() == 1:
            return
        for gi, g in enumerate(self.groups):
            for p in g:
                if p.requires_grad:
                    self.hooks.append(p.register_post_accumulate_grad_hook(lambda _p, gi=gi: self._arrived(gi)))
        self.overlap = True

    def _arrived(self, gi):
        self.count[gi] += 1
        need = self.expected[gi] * sum(1 for p in self.groups[gi] if p.requires_grad)
        if self.count[gi] == need and self.works[gi] is None:
            self._launch(gi)

    # ---- exchange -------------------------------------------------------------------
    def _ensure_flat(self):
        if self.flat is None:
            dev = self.groups[0][0].device
            self.flat = [[torch.empty(sum(p.numel() for p in b), dtype=torch.float32, device=dev) for b in bks]
                         for bks in self.buckets]

    def _launch(self, gi):
        self._ensure_flat()
        works = []
        for b, flat in zip(self.buckets[gi], self.flat[gi]):
            off = 0
            for p in b:
                n = p.numel()
                if p.grad is None:
                    flat[off:off + n].zero_()
                else:
                    flat[off:off + n].copy_(p.grad.reshape(-1))
                off += n
            works.append(dist.all_reduce(flat, op=dist.ReduceOp.SUM, async_op=True))
        self.works[gi] = works

    def __call__(self):
        w = world()
        if w == 1:
            return
        for gi in range(len(self.groups)):
            if self.works[gi] is None:
                self._launch(gi)
        for gi in range(len(self.groups)):
            for wk in self.works[gi]:
                wk.wait()
            for b, flat in zip(self.buckets[gi], self.flat[gi]):
                flat.mul_(1.0 / w)
                off = 0
                for p in b:
                    n = p.numel()
                    g = flat[off:off + n].view_as(p)
                    if p.grad is None:
                        p.grad = g.clone()
                    else:
                        p.grad.copy_(g)
                    off += n
        self.works = [None] * len(self.groups)
        self.count = [0] * len(self.groups)


def broadcast_buffers(modules, src=0):
    """Make every rank's BN running statistics equal to rank ``src``'s (DataParallel dev0 semantics)."""
    if world() == 1:
        return
    for m in modules:
        for b in m.buffers():
            dist.broadcast(b, src)
