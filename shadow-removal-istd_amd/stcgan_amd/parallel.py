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
Exchange per optimiser step (``BucketExchange``): each network's parameter gradients live in
one flat fp32 buffer (``FlatGrads``; every ``p.grad`` is a view of it, the weight-gradient kernels
write straight into those views), laid out in backward-completion order and cut into buckets of
~``bucket_mb``.  The engine reports each layer's gradients as it enqueues them (engine.GradWriter), and
a bucket's all-reduce is launched -- asynchronously, on a stream ordered after the streams that wrote
it -- the moment its last parameter is complete: the exchange of the deep layers runs while the
large-resolution layers of the same backward still compute.  The average is RCCL's ``AVG``
(gloo: sum, then a 1/world scale); there is no gather into or scatter out of a separate buffer.
Every rank runs the same program, so the collective sequence is identical on all ranks.
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
    t = torch.stack([values[k].double().reshape(()) for k in keys])  # (float64: the epoch sums)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    t.div_(world())
    return {k: t[i] for i, k in enumerate(keys)}


class FlatGrads:
    """The parameter gradients of one network in one flat fp32 buffer; ``view(p)`` is the slice that
    becomes ``p.grad``.  Parameters are laid out in reverse module order, which is the order their
    gradients are produced in (the generator's backward walks the up path from the outermost block
    inwards, then the down path outwards; the discriminator's from the logits layer down), so the
    buckets of a BucketExchange complete one after the other."""

    def __init__(self, params):
        self.params = list(params)
        dev = self.params[0].device
        self.spans = {}
        n = 0
        for p in reversed(self.params):
            self.spans[id(p)] = (n, p.numel())
            n += p.numel()
        self.numel = n
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.views = {}
        for p in self.params:
            o, k = self.spans[id(p)]
            self.views[id(p)] = self.flat[o:o + k].view(p.shape)

    def view(self, p):
        return self.views[id(p)]

    def owns(self, g, p):
        """Whether the tensor g is p's view of this buffer."""
        v = self.views.get(id(p))
        return v is not None and g is not None and g.data_ptr() == v.data_ptr() and g.shape == v.shape


def flat_grads(net):
    """The FlatGrads of a network module (created on first use on the parameters' device; dropped when
    the module moves: networks._HipNet._apply)."""
    fg = getattr(net, "_flat_grads", None)
    if fg is None:
        fg = FlatGrads(list(net.parameters()))
        net._flat_grads = fg
    return fg


def exchange_of(net):
    """The network's BucketExchange (``net.grad_exchange``, set by the trainer), re-made on the current flat
    buffer when the module moved since (networks._HipNet._apply drops the exchange bound to the old buffer and
    keeps its settings), so the ranks keep averaging its gradients after a ``.to()``."""
    ex = getattr(net, "grad_exchange", None)
    spec = getattr(net, "_exchange_spec", None)
    if ex is None and spec is not None:
        bucket_mb, active, on_complete, expected = spec
        ex = net.grad_exchange = BucketExchange(flat_grads(net), bucket_mb, active)
        ex.on_complete, ex.expected = on_complete, expected
        net._exchange_spec = None
    return ex


class BucketExchange:
    """Average one FlatGrads over all ranks, bucket by bucket, as the buckets complete.

    ``ready(params, stream)``: those parameters' gradients are enqueued (on ``stream``, or the current
    stream) and the backward no longer reads the parameters themselves; a bucket is complete once each of
    its parameters has been reported ``expected`` times (the discriminator's real and fake calls both
    write into its gradients in the D step).  A complete bucket is all-reduced (when ``active``) and then
    handed to ``on_complete(params, stream, work)`` -- the optimiser's per-bucket update (optim.Adam.overlap)
    -- when the average is final on the device (world size 1, or RCCL's in-collective AVG).  ``finish()``
    launches whatever is left, makes the current stream wait for every bucket and resets the counts."""

    def __init__(self, flat, bucket_mb=32, active=None):
        self.flat = flat
        # active: exchange even at world size 1 (tests drive the collective path on one GPU)
        self.active = (world() > 1) if active is None else bool(active)
        self.on_complete = None
        self.bucket_elems = max(1, int(bucket_mb * (1 << 20) // 4))
        self.ranges, self.members, self.bucket_of = [], [], {}
        cur, start, n = [], 0, 0
        for p in reversed(flat.params):
            o, k = flat.spans[id(p)]
            cur.append(id(p))
            n += k
            if n >= self.bucket_elems:
                self._cut(cur, start, o + k)
                cur, start, n = [], o + k, 0
        if cur:
            self._cut(cur, start, flat.numel)
        by_id = {id(p): p for p in flat.params}
        self.member_params = [[by_id[i] for i in m] for m in self.members]
        self.expected = 1
        self.launch_order = []  # bucket indices in launch order (diagnostics / tests)
        # diagnostics (scripts/exchange_timeline.py): when a list, every ready() call appends (parameter ids, event
        # recorded on the stream that wrote them) and finish() appends ("finish", event) -- also at world 1
        self.trace = None
        self.reset()

    def _cut(self, ids, a, e):
        b = len(self.ranges)
        self.ranges.append((a, e))
        self.members.append(list(ids))
        for i in ids:
            self.bucket_of[i] = b

    def reset(self):
        self.count = {}
        self.left = [len(m) for m in self.members]
        self.works = [None] * len(self.ranges)

    def _op(self):
        # RCCL/NCCL average in the collective (a power-of-two world scales exactly); gloo has no AVG
        return dist.ReduceOp.AVG if dist.get_backend() == "nccl" else dist.ReduceOp.SUM

    def _launch(self, b, stream=None):
        a, e = self.ranges[b]
        if stream is not None:  # a side stream that wrote part of the bucket: it also waits for the calling
            stream.wait_stream(torch.cuda.current_stream())  # stream, which wrote the rest
        if stream is None:
            self.works[b] = dist.all_reduce(self.flat.flat[a:e], op=self._op(), async_op=True)
        else:
            with torch.cuda.stream(stream):
                self.works[b] = dist.all_reduce(self.flat.flat[a:e], op=self._op(), async_op=True)
        self.launch_order.append(b)

    def ready(self, params, stream=None):
        if self.trace is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(stream if stream is not None else torch.cuda.current_stream())
            self.trace.append(([id(p) for p in params], ev))
        if not self.active and self.on_complete is None:
            return
        for p in params:
            c = self.count.get(id(p), 0) + 1
            self.count[id(p)] = c
            if c == self.expected:
                b = self.bucket_of[id(p)]
                self.left[b] -= 1
                if self.left[b] == 0:
                    if self.active:
                        self._launch(b, stream)
                    # gloo sums (the 1/world scale comes in finish): no early consumer then
                    if self.on_complete is not None and (not self.active or self._op() != dist.ReduceOp.SUM):
                        self.on_complete(self.member_params[b], stream, self.works[b])

    def check_order(self):
        """Debug check (tests, CPU gloo runs): every rank launched its buckets' collectives in the same order
        (the engine reports layers in autograd order; a divergence would pair different buckets in one
        collective).  Collective itself; raises on a mismatch.  Call before ``finish`` (which resets)."""
        if world() == 1:
            return
        mine = list(self.launch_order)
        allo = [None] * world()
        dist.all_gather_object(allo, mine)
        if any(o != allo[0] for o in allo):
            raise RuntimeError(f"BucketExchange: bucket launch order differs across ranks: {allo}")

    def finish(self):
        w = world()
        if self.trace is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.trace.append(("finish", ev))
        if not self.active:
            self.reset()
            return
        for b in range(len(self.ranges)):
            if self.works[b] is None:
                self._launch(b)
        for wk in self.works:
            wk.wait()
        if self._op() == dist.ReduceOp.SUM and w > 1:
            self.flat.flat.mul_(1.0 / w)
        self.reset()


class GradAllReduce:
    """Average the gradients of groups of ordinary autograd leaves over all ranks (for parameters that
    are not written by the engine): each group gets a FlatGrads whose zero-filled views are attached as
    the leaves' ``.grad`` (autograd accumulates into them in place) and a BucketExchange fed by
    post-accumulate-grad hooks.  ``__call__`` finishes the exchange (the engine's networks use
    FlatGrads/BucketExchange directly: engine.GradWriter)."""

    def __init__(self, groups, bucket_mb=32):
        self.flats = [FlatGrads(g) for g in groups]
        self.exchanges = [BucketExchange(f, bucket_mb) for f in self.flats]
        self.hooks = []
        for f, ex in zip(self.flats, self.exchanges):
            for p in f.params:
                if p.grad is not None:  # a gradient computed before the exchange was set up moves into the view
                    f.view(p).copy_(p.grad)
                p.grad = f.view(p)
                if p.requires_grad and world() > 1:
                    self.hooks.append(p.register_post_accumulate_grad_hook(lambda q, ex=ex, f=f: self._ready(f, ex, q)))

    @staticmethod
    def _ready(f, ex, q):
        # after a zero_grad(set_to_none=True) autograd accumulates into a fresh tensor, not the view: move it in
        if not f.owns(q.grad, q):
            v = f.view(q)
            v.copy_(q.grad)
            q.grad = v
        ex.ready([q])

    def enable_overlap(self):  # (hooks are registered at construction)
        pass

    def __call__(self):
        for ex in self.exchanges:
            ex.finish()
