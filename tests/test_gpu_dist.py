"""World-size-2 train step on ONE GPU (two processes, gloo over the device tensors): the
data-parallel exchange of parallel.GradAllReduce together with the side-stream step
(STCGAN.streams) and the engine-summed discriminator gradients (engine.WeightGradGroup).

Both ranks get the same batch, so the averaged gradient is (g + g) / 2 = g exactly and each
rank's post-step state must be bit-identical to a one-process step on that batch (with per-shard
BN each rank normalises the same shard).  The RCCL path is the same code with backend "nccl"
(one GPU per rank), which needs more than the one GPU a test box has."""
import io
import os
import socket
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, PKG_DIR, ROOT

pytestmark = pytest.mark.gpu

NETS = ("G1", "G2", "D1", "D2")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches():
    g = torch.Generator().manual_seed(21)
    return [tuple(torch.rand((4, c, 256, 256), generator=g) * 2 - 1 for c in (3, 1, 3)) for _ in range(2)]


def _trainer(loss_type):
    from stcgan_amd.stcgan import STCGAN
    torch.manual_seed(5)
    a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                              D_loss_fn="standard", D_loss_type=loss_type, ngf=16, dtype="bf16",
                              load_weights_g1=None, load_weights_g2=None, load_weights_d1=None,
                              load_weights_d2=None)
    return STCGAN(a)


def _steps(tr):
    for x, m, y in _batches():
        tr.train_step(x.cuda(), m.cuda(), y.cuda())
    torch.cuda.synchronize()
    return {n: {k: v.cpu() for k, v in getattr(tr, n).state_dict().items()} for n in NETS}


def _worker(rank, world, port, loss_type, out):
    import sys
    for p in (ROOT, PKG_DIR, GOLDEN):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        state = _steps(_trainer(loss_type))
        buf = io.BytesIO()
        torch.save(state, buf)
        out.put((rank, buf.getvalue()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("loss_type", ["normal", "rel_avg"])
def test_world2_same_batch_equals_one_process(loss_type):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, loss_type, q)) for r in range(2)]
    for p in procs:
        p.start()
    import queue
    import time
    got, t0 = {}, time.time()
    while len(got) < 2 and time.time() - t0 < 240:
        try:
            r, val = q.get(timeout=1)
            got[r] = val
        except queue.Empty:
            assert all(p.exitcode in (None, 0) for p in procs), [p.exitcode for p in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _steps(_trainer(loss_type))
    for r in (0, 1):
        st = torch.load(io.BytesIO(got[r]), weights_only=True)
        for n in NETS:
            for k, v in want[n].items():
                assert torch.equal(st[n][k], v), (r, n, k)
