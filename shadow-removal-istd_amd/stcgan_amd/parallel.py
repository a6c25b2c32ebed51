"""Data parallelism for the ST-CGAN step: one process per GPU, RCCL over xGMI.

Replaces ``nn.DataParallel`` (STCGAN/stcgan.py:53-59).  Semantics kept from the
reference:
  * every replica computes with the same weights: DataParallel broadcasts dev0's
    parameters before each forward; here rank 0's initial parameters and buffers
    are broadcast once (``broadcast_state``) and the averaged gradients keep the
    ranks identical afterwards;
  * BatchNorm statistics are per shard (each rank normalises its own slice) and the
    running statistics that matter are rank 0's (DataParallel keeps dev0's
    replica): before an eval-mode pass every rank takes rank 0's buffers
    (``broadcast_buffers``), as the replicas of an eval-mode DataParallel forward do;
  * the losses see the global batch: the mean losses are means of equal shards, so
    the per-rank means average to the global one; the relativistic batch means
    ``C.mean(dim=0)`` of the rel_avg loss (STCGAN/stcgan.py:240-250, 280-290) are
    all-reduced inside the graph (``global_mean0``); the epoch loss sums fed to
    ReduceLROnPlateau (STCGAN/stcgan.py:314-315) are all-reduced (``average_scalars``)
    so every rank's scheduler sees the same (global) values.
Exchange per optimiser step: one all-reduce of the gradients per network (sum,
then scaled by 1/world).

Overlap: every network's gradients arrive in one autograd node (engine.NetFn),
so a post-accumulate-grad hook counts arrivals per network and launches that
network's bucketed all-reduce asynchronously the moment its last gradient lands
-- G2's 218 MB exchange runs while G1's backward still computes.  Groups are
launched in index order on every rank (a completed group waits for the groups
before it), so the collective sequence is identical across ranks whatever the
hook timing.  ``__call__`` launches whatever did not fire, waits, and scatters
the averages back.
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


def broadcast_state(modules, src=0):
    """Every rank takes rank ``src``'s parameters and buffers (DataParallel replicates dev0's
    module into every replica, STCGAN/stcgan.py:53-59)."""
    if world() == 1:
        return
    with torch.no_grad():
        for m in modules:
            for t in list(m.parameters()) + list(m.buffers()):
                dist.broadcast(t.data, src)
            # the in-place write through .data does not bump the parameters' versions: drop any packed
            # operands made from the pre-broadcast values
            if getattr(m, "_pack_cache", None):
                from . import ops
                m._pack_cache.clear()
                ops.invalidate_packs()


def broadcast_buffers(modules, src=0):
    """Make every rank's BN running statistics equal to rank ``src``'s (DataParallel dev0 semantics)."""
    if world() == 1:
        return
    for m in modules:
        for b in m.buffers():
            dist.broadcast(b, src)


class _AllReduceAvg(torch.autograd.Function):
    """y = mean over ranks of x.  Backward: the gradient of a rank's input collects the
    gradients every rank's loss sends into the shared mean: mean over ranks again (the
    parameter gradients are averaged afterwards, so a factor world is folded in)."""

    @staticmethod
    def forward(ctx, x):
        y = x.detach().clone()
        dist.all_reduce(y, op=dist.ReduceOp.SUM)
        return y.div_(world())

    @staticmethod
    def backward(ctx, g):
        g = g.detach().clone().contiguous()
        dist.all_reduce(g, op=dist.ReduceOp.SUM)
        return g.div_(world())


def global_mean0(x):
    """``x.mean(dim=0)`` over the GLOBAL batch (all ranks' equal shards), differentiable.
    What ``C.mean(dim=0)`` computes on DataParallel's gathered output (STCGAN/stcgan.py:240-250)."""
    m = x.mean(dim=0)
    if world() == 1:
        return m
    return _AllReduceAvg.apply(m)


def average_scalars(values):
    """Average a dict of device scalars over the ranks (one collective); returns a new dict."""
    if world() == 1:
        return dict(values)
    keys = list(values)
    t = torch.stack([values[k].float().reshape(()) for k in keys])
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    t.div_(world())
    return {k: t[i] for i, k in enumerate(keys)}


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
        self.ready = [False] * len(self.groups)
        self.hooks = []
        self.overlap = False
        # streams the gradients of each group were accumulated on (autograd runs a leaf's
        # AccumulateGrad, and so the hook, on the stream of the backward that produced it; the
        # discriminators' backwards run on side streams): the exchange waits for all of them
        self.arrival_streams = [dict() for _ in self.groups]
        self.cuda = bool(self.groups) and bool(self.groups[0]) and self.groups[0][0].is_cuda

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
        if self.cuda:
            st = torch.cuda.current_stream()
            self.arrival_streams[gi].setdefault(st.cuda_stream, st)
        need = self.expected[gi] * sum(1 for p in self.groups[gi] if p.requires_grad)
        if self.count[gi] == need:
            self.ready[gi] = True
            # launch in index order: group gi only after groups 0..gi-1 (same sequence on every rank)
            for gj in range(len(self.groups)):
                if self.works[gj] is not None:
                    continue
                if not self.ready[gj]:
                    break
                self._launch(gj)

    # ---- exchange -------------------------------------------------------------------
    def _ensure_flat(self):
        if self.flat is None:
            dev = self.groups[0][0].device
            self.flat = [[torch.empty(sum(p.numel() for p in b), dtype=torch.float32, device=dev) for b in bks]
                         for bks in self.buckets]

    def _launch(self, gi):
        self._ensure_flat()
        # the launching hook may run on another group's stream (a group completing early waits
        # for the groups before it): order the gather after every stream this group's gradients
        # were written on
        if self.arrival_streams[gi]:
            cur = torch.cuda.current_stream()
            for key, st in self.arrival_streams[gi].items():
                if key != cur.cuda_stream:
                    cur.wait_stream(st)
            self.arrival_streams[gi].clear()
        works = []
        for b, flat in zip(self.buckets[gi], self.flat[gi]):
            grads = [p.grad.reshape(-1) if p.grad is not None else None for p in b]
            if all(g is not None for g in grads):
                torch.cat(grads, out=flat)  # one gather kernel per bucket
            else:
                off = 0
                for p, g in zip(b, grads):
                    n = p.numel()
                    if g is None:
                        flat[off:off + n].zero_()
                    else:
                        flat[off:off + n].copy_(g)
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
                for p in b:
                    if p.grad is None:
                        p.grad = torch.empty_like(p)
                parts = [s.view_as(p) for s, p in zip(torch.split(flat, [p.numel() for p in b]), b)]
                torch._foreach_copy_([p.grad for p in b], parts)  # one multi-tensor launch per bucket
        self.works = [None] * len(self.groups)
        self.count = [0] * len(self.groups)
        self.ready = [False] * len(self.groups)
