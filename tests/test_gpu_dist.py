"""Data parallelism on the GPU: one process per rank, each rank training on its OWN shard.

The reference's multi-GPU path is nn.DataParallel (STCGAN/stcgan.py:53-59): every network call
scatters the batch over the devices, each replica normalises its own shard (per-shard BatchNorm), only
device 0's replica keeps its running-statistics update, and the losses see the gathered batch.  Here
that is one process per GPU with the gradients of each network averaged bucket by bucket while its
backward runs (parallel.BucketExchange, fed by engine.GradWriter).

* ``test_world2_shards_match_dataparallel_oracle``: two ranks (two processes sharing the test box's one
  GPU, gloo over the device tensors), DIFFERENT shards of each global batch, two train steps; every
  parameter of both ranks (bit-identical to each other) and rank 0's BatchNorm buffers against the CPU
  oracle running the reference's DataParallel semantics on the whole global batch
  (oracle.stcgan_ref.OracleSTCGAN(shards=2)), at the fp32 tolerances of the reference run_epoch test.
* ``test_world2_same_batch_equals_one_process``: both ranks on the same batch must equal one process
  bit for bit (the average of two equal gradients is that gradient).
* ``test_rccl_exchange_world1``: the RCCL backend (torch "nccl") on one rank with the exchange forced on:
  the bucketed all-reduce (ReduceOp.AVG) runs inside the backward and leaves the step bit-identical.
The 8-GPU RCCL run itself is the driver's (bench.py --gpus 8)."""
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
NET_SEED = {"G1": 11, "G2": 12, "D1": 13, "D2": 14}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_batches(n=2, bs=4, seed=2100):
    from fixture_init import pm_one, uniform
    return [(uniform((bs, 3, 256, 256), seed + 10 * i), pm_one((bs, 1, 256, 256), seed + 10 * i + 1),
             uniform((bs, 3, 256, 256), seed + 10 * i + 2)) for i in range(n)]


def _trainer(loss_type, ngf, dtype, family):
    from fixture_init import fixture_state
    from stcgan_amd.stcgan import STCGAN
    if os.environ.get("STC_TEST_SPLITK_INLAUNCH") == "0":  # (diagnostic A/B of the in-launch split-K)
        from stcgan_amd import ops
        ops.set_splitk_inlaunch(False)
    torch.manual_seed(5)
    a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                              D_loss_fn="standard", D_loss_type=loss_type, ngf=ngf, dtype=dtype,
                              load_weights_g1=None, load_weights_g2=None, load_weights_d1=None,
                              load_weights_d2=None)
    tr = STCGAN(a)
    if family is not None:
        for name in NETS:
            net = getattr(tr, name)
            net.load_state_dict(fixture_state(net.state_dict(), NET_SEED[name], family))
    return tr


def _state(tr):
    torch.cuda.synchronize()
    return {n: {k: v.detach().cpu().clone() for k, v in getattr(tr, n).state_dict().items()} for n in NETS}


def _paths():
    import sys
    for p in (ROOT, PKG_DIR, GOLDEN):
        if p not in sys.path:
            sys.path.insert(0, p)


def _worker(rank, world, port, cfg, out):
    _paths()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        loss_type, ngf, dtype, family, same = cfg
        tr = _trainer(loss_type, ngf, dtype, family)
        from stcgan_amd import engine
        assert tr.streams and engine.WGRAD_OVERLAP  # (the side lanes and weight-gradient streams are on)
        launched = {}
        for x, m, y in _global_batches():
            if not same:  # this rank's shard of the global batch
                b = x.shape[0] // world
                x, m, y = (t[rank * b:(rank + 1) * b] for t in (x, m, y))
            tr.train_step(x.cuda(), m.cuda(), y.cuda())
            # every rank launched each network's bucket collectives in the same order (raises otherwise): the
            # engine reports buckets in autograd order, whatever the lanes' enqueue timing
            for n in NETS:
                ex = getattr(tr, n).grad_exchange
                ex.check_order()
                launched[n] = len(ex.launch_order)
        assert all(v > 0 for v in launched.values()), launched
        buf = io.BytesIO()
        torch.save(_state(tr), buf)  # bytes, not shared-memory tensors: the worker may exit first
        out.put((rank, buf.getvalue()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run_world(cfg, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time
    got, t0 = {}, time.time()
    while len(got) < world and time.time() - t0 < 240:
        try:
            r, val = q.get(timeout=1)
            got[r] = val
        except queue.Empty:
            assert all(p.exitcode in (None, 0) for p in procs), [p.exitcode for p in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return {r: torch.load(io.BytesIO(v), weights_only=True) for r, v in got.items()}


@pytest.mark.parametrize("loss_type", ["normal", "rel_avg"])
def test_world2_shards_match_dataparallel_oracle(loss_type):
    _paths()
    from fixture_init import fixture_state
    from oracle import stcgan_ref as ref
    got = _run_world((loss_type, 8, "fp32", "ref", False))
    for n in NETS:  # the ranks hold the same parameters (the all-reduce leaves every rank the same average)
        for k, v in got[0][n].items():
            if not k.endswith(("running_mean", "running_var", "num_batches_tracked")):
                assert torch.equal(v, got[1][n][k]), (n, k)
    templ = {"G1": ref.generator_state_template(3, 1, 8), "G2": ref.generator_state_template(4, 3, 8),
             "D1": ref.discriminator_state_template(4, 8), "D2": ref.discriminator_state_template(7, 8)}
    orc = ref.OracleSTCGAN({n: fixture_state(templ[n], NET_SEED[n], "ref") for n in NETS}, loss_type=loss_type,
                           shards=2)
    orc.run_epoch([([], x, m, y) for x, m, y in _global_batches()], training=True)
    worst = 0.0
    for n in NETS:
        for k, v in got[0][n].items():
            w = orc.st[n][k].detach()
            if not v.is_floating_point():
                assert torch.equal(v, w), (n, k)
                continue
            # the tolerance of tests/test_gpu_model.py::test_run_epoch_vs_golden (two iterations)
            err = (v.double() - w.double()).abs()
            lim = 5e-5 + 1e-4 * w.double().abs()
            worst = max(worst, float((err / lim).max()))
            assert bool((err <= lim).all()), (n, k, float(err.max()))
    print(f"world-2 shards vs DataParallel oracle [{loss_type}]: worst error / tolerance {worst:.3f}")


def test_world2_same_batch_equals_one_process():
    got = _run_world(("normal", 16, "bf16", None, True))
    want = _state(_run_one(("normal", 16, "bf16", None)))
    for r in (0, 1):
        for n in NETS:
            for k, v in want[n].items():
                assert torch.equal(got[r][n][k], v), (r, n, k)


def _run_one(cfg, exchange=False):
    loss_type, ngf, dtype, family = cfg
    tr = _trainer(loss_type, ngf, dtype, family)
    if exchange:
        from stcgan_amd import parallel
        for n in NETS:
            net = getattr(tr, n)
            net.grad_exchange = parallel.BucketExchange(parallel.flat_grads(net), bucket_mb=1, active=True)
    for x, m, y in _global_batches():
        tr.train_step(x.cuda(), m.cuda(), y.cuda())
    return tr


def _rccl_worker(port, out):
    _paths()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        cfg = ("normal", 16, "bf16", "ref")
        tr = _run_one(cfg, exchange=True)
        launched = sum(len(getattr(tr, n).grad_exchange.launch_order) for n in NETS)
        st = _state(tr)
        ref_st = _state(_run_one(cfg))
        bad = [(n, k) for n in NETS for k in st[n] if not torch.equal(st[n][k], ref_st[n][k])]
        out.put((dist.get_backend(), launched, bad))
    finally:
        dist.destroy_process_group()


def test_rccl_exchange_world1():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    backend, launched, bad = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert backend == "nccl" and launched > 8, (backend, launched)
    assert not bad, bad[:8]
