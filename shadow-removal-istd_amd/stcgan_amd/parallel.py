"""Data parallelism for the ST-CGAN step: one process per GPU, RCCL over xGMI.

Replaces ``nn.DataParallel`` (STCGAN/stcgan.py:53-59).  Semantics kept from the
reference: BatchNorm statistics are per shard (each rank normalises its own
slice), the loss is the mean over the global batch (= the average of the
per-rank means for equal shards), and the running statistics that matter are
rank 0's (DataParallel keeps dev0's replica).  Exchange per optimiser step:
one bucketed all-reduce of the gradients (sum, then scaled by 1/world).
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
    """Average the .grad of ``params`` over all ranks with flat fp32 buckets.

    Buckets are ~``bucket_mb`` MB (sized for per-link ring bandwidth on xGMI:
    a few large collectives rather than many small ones).  Grads are copied
    into persistent flat buffers, reduced asynchronously bucket by bucket, and
    copied back."""

    def __init__(self, params, bucket_mb=64):
        self.params = [p for p in params]
        self.bucket_elems = int(bucket_mb * (1 << 20) // 4)
        self.buckets = []
        cur, n = [], 0
        for p in self.params:
            cur.append(p)
            n += p.numel()
            if n >= self.bucket_elems:
                self.buckets.append(cur)
                cur, n = [], 0
        if cur:
            self.buckets.append(cur)
        self.flat = None

    def __call__(self):
        w = world()
        if w == 1:
            return
        if self.flat is None:
            dev = self.params[0].device
            self.flat = [torch.empty(sum(p.numel() for p in b), dtype=torch.float32, device=dev)
                         for b in self.buckets]
        works = []
        for b, flat in zip(self.buckets, self.flat):
            off = 0
            for p in b:
                n = p.numel()
                if p.grad is None:
                    flat[off:off + n].zero_()
                else:
                    flat[off:off + n].copy_(p.grad.reshape(-1))
                off += n
            works.append(dist.all_reduce(flat, op=dist.ReduceOp.SUM, async_op=True))
        for b, flat, wk in zip(self.buckets, self.flat, works):
            wk.wait()
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


def broadcast_buffers(modules, src=0):
    """Make every rank's BN running statistics equal to rank ``src``'s (DataParallel dev0 semantics)."""
    if world() == 1:
        return
    for m in modules:
        for b in m.buffers():
            dist.broadcast(b, src)
