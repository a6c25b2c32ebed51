"""World-size-2 gloo tests of the data-parallel layer (parallel.py), on CPU.

Checks the reference's DataParallel semantics that the RCCL path keeps
(STCGAN/stcgan.py:53-59):
  * with per-shard BN, the averaged per-rank gradient of the per-rank mean loss
    equals the gradient of the global-batch mean loss (equal shards);
  * the rel_avg loss (STCGAN/stcgan.py:240-250) uses C.mean(dim=0) over the GLOBAL
    batch -- ``global_mean0`` -- and its gradients match the single-process loss;
  * ranks that initialise from different seeds hold rank 0's weights after
    ``broadcast_state`` (DataParallel replicates dev0's module);
  * the epoch loss sums fed to ReduceLROnPlateau are the global ones on every rank;
  * each network's flat gradient buffer is exchanged bucket by bucket as the buckets complete.
The networks here are the CPU oracle (test infrastructure) -- only the exchange
logic is under test.
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
    # two groups, each one flat buffer (the leaves' .grad are views of it) cut into several buckets; the
    # net is used twice in the graph (real + fake) but autograd sums the uses before accumulating, so each
    # parameter's hook fires once per backward
    sync = parallel.GradAllReduce([plist[:half], plist[half:]], bucket_mb=0.002)
    assert all(len(ex.ranges) > 1 for ex in sync.exchanges)  # several buckets per group
    assert all(sync.flats[i].owns(p.grad, p) for i, grp in enumerate((plist[:half], plist[half:])) for p in grp)
    sl = slice(rank * 2, (rank + 1) * 2)
    out_a = ref.discriminator_forward(params, x[sl], True)
    out_b = ref.discriminator_forward(params, z[sl], True)
    loss = (((out_a - 1.0) ** 2).mean() + (out_b ** 2).mean()) * 0.5
    loss.backward()
    assert all(w is not None for ex in sync.exchanges for w in ex.works)  # launched from the backward hooks
    sync()
    assert all(w is None for ex in sync.exchanges for w in ex.works) and all(not ex.count for ex in sync.exchanges)
    if rank == 0:
        import io
        buf = io.BytesIO()
        torch.save([p.grad.clone() for p in plist], buf)  # bytes: the worker may exit before the parent reads
        out.put(buf.getvalue())
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
    import io
    got = torch.load(io.BytesIO(got), weights_only=True)
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


def _run_world(target, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time
    got, t0 = {}, time.time()
    while len(got) < world and time.time() - t0 < 300:
        try:
            r, val = q.get(timeout=1)
            got[r] = val
        except queue.Empty:
            assert all(p.exitcode in (None, 0) for p in procs), [p.exitcode for p in procs]
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    return got


def _rel_avg_loss(params, x, z, mean0):
    """The reference's rel_avg D1 loss on a (real, fake) pair (STCGAN/stcgan.py:240-245)."""
    from oracle import stcgan_ref as ref
    c_real = ref.discriminator_forward(params, x, True)
    c_fake = ref.discriminator_forward(params, z, True)
    return (ref.adversarial_loss(c_fake - mean0(c_real), False)
            + ref.adversarial_loss(c_real - mean0(c_fake), True)) * 0.5


def _worker_semantics(rank, world, port, out):
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
    res = {}
    # (1) broadcast_state: different seeds per rank -> rank 0's weights everywhere
    torch.manual_seed(100 + rank)
    net = torch.nn.Sequential(torch.nn.Conv2d(4, 8, 4, 2, 1), torch.nn.BatchNorm2d(8))
    with torch.no_grad():
        net[1].running_mean.normal_()
    parallel.broadcast_state([net])
    res["state"] = {k: v.clone() for k, v in net.state_dict().items()}
    # (2) rel_avg with the global batch mean: gradients averaged over ranks
    st = fixture_state(ref.discriminator_state_template(4, 8), 13, "one")
    params = {k: v.clone().requires_grad_(not ref._is_buffer(k)) for k, v in st.items()}
    x = uniform((4, 4, 64, 64), 7)
    z = uniform((4, 4, 64, 64), 8)
    sl = slice(rank * 2, (rank + 1) * 2)
    loss = _rel_avg_loss(params, x[sl], z[sl], parallel.global_mean0)
    loss.backward()
    plist = [v for k, v in params.items() if v.requires_grad]
    sync = parallel.GradAllReduce([plist])
    sync()
    res["rel_avg_grads"] = [p.grad.clone() for p in plist]
    res["rel_avg_loss"] = parallel.average_scalars({"l": loss.detach()})["l"].clone()
    # (3) scheduler inputs: every rank sees the global sums
    acc = {"G": torch.tensor(float(rank + 1)), "D": torch.tensor(10.0 * (rank + 1))}
    avg = parallel.average_scalars(acc)
    res["sched"] = (float(avg["G"]), float(avg["D"]))
    # (4) engine-style exchange: gradients written into the flat views and reported per layer; with
    # expected = 2 (the discriminator's real and fake calls) a bucket launches on its second report, in
    # completion order (b's bucket before a's: b is later in module order, so earlier in the flat buffer)
    a = torch.zeros(3, requires_grad=True)
    b = torch.zeros(5, requires_grad=True)
    fg = parallel.FlatGrads([a, b])
    ex = parallel.BucketExchange(fg, bucket_mb=1e-6)  # one parameter per bucket
    ex.expected = 2
    fg.view(a).fill_(2.0 * (rank + 1))
    fg.view(b).fill_(float(rank + 1))
    ex.ready([b])
    held = list(ex.launch_order)
    ex.ready([b])
    ex.ready([a])
    ex.ready([a])
    order = list(ex.launch_order)
    ex.finish()
    res["order"] = (held, order, fg.view(a).clone(), fg.view(b).clone(), [fg.spans[id(a)], fg.spans[id(b)]])
    # (5) a ragged final batch of 5 (shards 3 + 2, data.shard_bounds): each rank's means weighted by its share
    # (stcgan.batch_weight) average to the global-batch means the reference logs (STCGAN/stcgan.py:256-262)
    from stcgan_amd import data, stcgan
    per_sample = torch.tensor([0.5, 1.25, -2.0, 4.0, 0.75])
    c_out = torch.arange(5 * 4, dtype=torch.float32).reshape(5, 1, 2, 2) / 7.0
    lo, hi = data.shard_bounds(5, rank, world)
    acc = {k: torch.zeros((), dtype=torch.float64) for k in ("D", "D1_real", "D1_fake", "D2_real", "D2_fake")}
    w = stcgan.batch_weight(hi - lo, 5, world)
    stcgan.accumulate(acc, {"D": per_sample[lo:hi].mean()}, [c_out[lo:hi]] * 4, w)
    res["ragged"] = ((lo, hi), {k: float(v) for k, v in parallel.average_scalars(acc).items()})
    # (5b) ... and its gradients: each rank back-propagates its shard mean scaled by the same weight
    # (stcgan.weighted_loss), so the equal-weight rank average is the global-batch mean's gradient
    wv = torch.zeros(3, requires_grad=True)
    feats = torch.arange(15, dtype=torch.float32).reshape(5, 3) / 4.0 - 1.0
    shard_mean = ((feats[lo:hi] * (wv + 0.5)).sum(1) ** 2).mean()
    stcgan.weighted_loss(shard_mean, w).backward()
    parallel.GradAllReduce([[wv]])()
    res["ragged_grad"] = wv.grad.clone()
    # (6) GradAllReduce across a set_to_none zero_grad: autograd's fresh gradients are moved into the views
    q = torch.zeros(4, requires_grad=True)
    sync2 = parallel.GradAllReduce([[q]])
    for it in range(2):
        q.grad = None  # (optimizer.zero_grad(set_to_none=True))
        (q * float(rank + 1 + it)).sum().backward()
        sync2.exchanges[0].check_order()
        sync2()
    res["zero_grad"] = (q.grad.clone(), sync2.flats[0].owns(q.grad, q))
    import io
    buf = io.BytesIO()
    torch.save(res, buf)  # bytes, not shared-memory tensors: the worker exits before the parent reads
    out.put((rank, buf.getvalue()))
    dist.barrier()
    dist.destroy_process_group()


def test_dataparallel_semantics_world2():
    import sys
    for p in (ROOT, PKG_DIR, GOLDEN):
        if p not in sys.path:
            sys.path.insert(0, p)
    from fixture_init import fixture_state, uniform
    from oracle import stcgan_ref as ref
    import io
    got = _run_world(_worker_semantics)
    r0, r1 = (torch.load(io.BytesIO(got[r]), weights_only=True) for r in (0, 1))
    for k in r0["state"]:
        assert torch.equal(r0["state"][k], r1["state"][k]), k
    # single process, global batch of 4, per-shard BN (two shards), global C.mean(dim=0)
    st = fixture_state(ref.discriminator_state_template(4, 8), 13, "one")
    params = {k: v.clone().requires_grad_(not ref._is_buffer(k)) for k, v in st.items()}
    x = uniform((4, 4, 64, 64), 7)
    z = uniform((4, 4, 64, 64), 8)
    cr = torch.cat([ref.discriminator_forward(params, x[i * 2:(i + 1) * 2], True) for i in range(2)])
    cf = torch.cat([ref.discriminator_forward(params, z[i * 2:(i + 1) * 2], True) for i in range(2)])
    loss = (ref.adversarial_loss(cf - cr.mean(dim=0), False) + ref.adversarial_loss(cr - cf.mean(dim=0), True)) * 0.5
    loss.backward()
    want = [v.grad for k, v in params.items() if v.requires_grad]
    for r in (r0, r1):
        assert abs(float(r["rel_avg_loss"]) - float(loss)) <= 1e-6 * abs(float(loss)) + 1e-7
        for g, w in zip(r["rel_avg_grads"], want):
            assert torch.allclose(g, w, atol=1e-6, rtol=1e-5)
        assert r["sched"] == (1.5, 15.0)
        held, order, ga, gb, spans = r["order"]
        assert spans == [(5, 3), (0, 5)]  # reverse module order: b first
        assert held == [] and order == [0, 1]
        assert torch.equal(ga, torch.full((3,), 3.0)) and torch.equal(gb, torch.full((5,), 1.5))
        # ragged final batch: the logged values are the global-batch means
        per_sample = torch.tensor([0.5, 1.25, -2.0, 4.0, 0.75], dtype=torch.float64)
        c_out = torch.arange(5 * 4, dtype=torch.float32).reshape(5, 1, 2, 2) / 7.0
        bounds, vals = r["ragged"]
        assert abs(vals["D"] - float(per_sample.mean())) < 1e-6  # (fp32 per-rank means)
        assert abs(vals["D1_fake"] - float(c_out.double().mean())) < 1e-6
        # ... and the gradient is the global-batch mean's (DataParallel), not the mean of the shard means
        wv = torch.zeros(3, requires_grad=True)
        feats = torch.arange(15, dtype=torch.float32).reshape(5, 3) / 4.0 - 1.0
        ((feats * (wv + 0.5)).sum(1) ** 2).mean().backward()
        assert torch.allclose(r["ragged_grad"], wv.grad, atol=1e-6, rtol=1e-5), (r["ragged_grad"], wv.grad)
        # second backward after zero_grad(set_to_none): still averaged over ranks ((1+2)/2 + 1)
        g, owned = r["zero_grad"]
        assert owned and torch.equal(g, torch.full((4,), 2.5))
    assert r0["ragged"][0] == (0, 3) and r1["ragged"][0] == (3, 5)
