"""World-size-2 gloo test of the data-parallel gradient exchange (parallel.py), on CPU.

Checks the reference's DataParallel semantics that the RCCL path keeps: with
per-shard BN, the averaged per-rank gradient of the per-rank mean loss equals
the gradient of the global-batch mean loss (equal shards).  The networks here
are the CPU oracle (test infrastructure) -- only the exchange logic is under test.
"""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, PKG_DIR, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    for p in (ROOT, PKG_DIR, GOLDEN):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from fixture_init import fixture_state, uniform
    from oracle import stcgan_ref as ref
    from stcgan_amd import parallel
    st = fixture_state(ref.discriminator_state_template(4, 8), 13, "one")
    params = {k: v.clone().requires_grad_(not ref._is_buffer(k)) for k, v in st.items()}
    x = uniform((4, 4, 64, 64), 7)  # global batch 4, shard by rank
    z = uniform((4, 4, 64, 64), 8)
    plist = [v for k, v in params.items() if v.requires_grad]
    half = len(plist) // 2
    # two groups; the net is used twice in the graph (real + fake) but autograd sums the
    # uses before accumulating, so each parameter's hook fires once per backward
    sync = parallel.GradAllReduce([plist[:half], plist[half:]], bucket_mb=0.002)
    assert all(len(b) > 1 for b in sync.buckets)  # several buckets per group
    sync.enable_overlap()
    sl = slice(rank * 2, (rank + 1) * 2)
    out_a = ref.discriminator_forward(params, x[sl], True)
    out_b = ref.discriminator_forward(params, z[sl], True)
    loss = (((out_a - 1.0) ** 2).mean() + (out_b ** 2).mean()) * 0.5
    loss.backward()
    assert all(w is not None for w in sync.works)  # launched from the backward hooks
    sync()
    assert sync.works == [None, None] and sync.count == [0, 0]
    if rank == 0:
        out.put([p.grad.clone() for p in plist])
    dist.barrier()
    dist.destroy_process_group()


def test_grad_allreduce_matches_global_batch():
    import sys
    for p in (ROOT, PKG_DIR, GOLDEN):
        if p not in sys.path:
            sys.path.insert(0, p)
    from fixture_init import fixture_state, uniform
    from oracle import stcgan_ref as ref
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    import queue
    import time
    got, t0 = None, time.time()
    while got is None and time.time() - t0 < 300:
        try:
            got = q.get(timeout=1)
        except queue.Empty:
            assert all(p.exitcode in (None, 0) for p in procs), [p.exitcode for p in procs]
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    # single-process reference: per-shard BN (two forwards), loss = mean over the global batch
    st = fixture_state(ref.discriminator_state_template(4, 8), 13, "one")
    params = {k: v.clone().requires_grad_(not ref._is_buffer(k)) for k, v in st.items()}
    x = uniform((4, 4, 64, 64), 7)
    z = uniform((4, 4, 64, 64), 8)
    loss = 0
    for i in range(2):
        sl = slice(i * 2, (i + 1) * 2)
        out_a = ref.discriminator_forward(params, x[sl], True)
        out_b = ref.discriminator_forward(params, z[sl], True)
        loss = loss + (((out_a - 1.0) ** 2).mean() + (out_b ** 2).mean()) * 0.5 / 2
    loss.backward()
    want = [v.grad for k, v in params.items() if v.requires_grad]
    for g, w in zip(got, want):
        assert torch.allclose(g, w, atol=1e-6, rtol=1e-5)
