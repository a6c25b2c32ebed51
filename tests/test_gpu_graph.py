"""The train step captured as one HIP graph (STCGAN.capture) and replayed must be the eager step, bit
for bit: same kernels, same memory contents, the side-stream branches and the device-resident Adam step
count included.  Two trainers from one initial state: eager steps on one, capture + replays on the
other; every parameter, BatchNorm buffer and Adam moment must agree exactly after each replay, and the
optimiser's host-side step counts must come back right (state_dict)."""
import types

import pytest
import torch

pytestmark = pytest.mark.gpu

NETS = ("G1", "G2", "D1", "D2")


def _trainer(dtype, ngf, loss_type):
    from stcgan_amd.stcgan import STCGAN
    torch.manual_seed(7)
    a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                              D_loss_fn="standard", D_loss_type=loss_type, ngf=ngf, dtype=dtype,
                              load_weights_g1=None, load_weights_g2=None, load_weights_d1=None,
                              load_weights_d2=None)
    return STCGAN(a)


def _state(tr):
    torch.cuda.synchronize()
    st = {n: {k: v.detach().clone() for k, v in getattr(tr, n).state_dict().items()} for n in NETS}
    for oname in ("optim_G", "optim_D"):
        o = getattr(tr, oname)
        o.sync_steps()
        st[oname] = [(float(o.state[p]["step"]), o.state[p]["exp_avg"].clone(), o.state[p]["exp_avg_sq"].clone())
                     for g in o.param_groups for p in g["params"]]
    return st


def _same(a, b):
    bad = []
    for n in NETS:
        for k in a[n]:
            if not torch.equal(a[n][k], b[n][k]):
                bad.append((n, k))
    for oname in ("optim_G", "optim_D"):
        for i, (x, y) in enumerate(zip(a[oname], b[oname])):
            if x[0] != y[0] or not torch.equal(x[1], y[1]) or not torch.equal(x[2], y[2]):
                bad.append((oname, i))
    return bad


@pytest.mark.parametrize("dtype,ngf,loss_type", [("bf16", 64, "normal"), ("fp32", 16, "rel_avg")])
def test_captured_step_is_bit_identical(dtype, ngf, loss_type):
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    B = 4
    x = torch.rand((B, 3, 256, 256), generator=g, device="cuda") * 2 - 1
    m = (torch.rand((B, 1, 256, 256), generator=g, device="cuda") < 0.5).float() * 2 - 1
    y = torch.rand((B, 3, 256, 256), generator=g, device="cuda") * 2 - 1
    eager = _trainer(dtype, ngf, loss_type)
    graphed = _trainer(dtype, ngf, loss_type)
    replay = graphed.capture(x, m, y, warmup=1)  # 3 eager steps inside (warm-up + two in device-step mode)
    for _ in range(3):
        eager.train_step(x, m, y)
    assert not _same(_state(eager), _state(graphed))
    for i in range(3):
        eager.train_step(x, m, y)
        replay()
        bad = _same(_state(eager), _state(graphed))
        assert not bad, (i, bad[:8])
    # new batch contents in place: the replay reads them
    x.copy_(torch.rand((B, 3, 256, 256), generator=g, device="cuda") * 2 - 1)
    eager.train_step(x, m, y)
    replay()
    assert not _same(_state(eager), _state(graphed))
    assert float(graphed.optim_G.state[next(graphed.G1.parameters())]["step"]) == 7.0


def test_general_path_step_after_replays():
    """Replays advance only the device step counters; an eager step that then takes the optimiser's general path
    (here: every packed operand re-registered, ops.invalidate_packs) must continue from the device count, and so
    must the replay after it (the host count used to be stale there)."""
    from stcgan_amd import ops
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    B = 2
    x = torch.rand((B, 3, 256, 256), generator=g, device="cuda") * 2 - 1
    m = (torch.rand((B, 1, 256, 256), generator=g, device="cuda") < 0.5).float() * 2 - 1
    y = torch.rand((B, 3, 256, 256), generator=g, device="cuda") * 2 - 1
    eager = _trainer("bf16", 16, "normal")
    graphed = _trainer("bf16", 16, "normal")
    replay = graphed.capture(x, m, y, warmup=1)  # 3 eager steps inside
    for _ in range(3):
        eager.train_step(x, m, y)
    for _ in range(2):  # no sync_steps between the replays and the eager step below
        eager.train_step(x, m, y)
        replay()
    ops.invalidate_packs()  # both trainers' next step: the general Adam path
    eager.train_step(x, m, y)
    graphed.train_step(x, m, y)
    bad = _same(_state(eager), _state(graphed))
    assert not bad, bad[:8]
    eager.train_step(x, m, y)
    replay()
    bad = _same(_state(eager), _state(graphed))
    assert not bad, bad[:8]
    assert float(graphed.optim_D.state[next(graphed.D1.parameters())]["step"]) == 7.0


def test_replay_after_optimizer_state_load():
    """An optimiser state loaded into a captured trainer (a checkpoint resume) must reach the replay: the loaded
    moments are copied into the moment buffers the graph's pointer tables hold (torch's
    load_state_dict swapped in new tensors, and the replay kept updating the old ones)."""
    import copy
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    B = 2
    x = torch.rand((B, 3, 256, 256), generator=g, device="cuda") * 2 - 1
    m = (torch.rand((B, 1, 256, 256), generator=g, device="cuda") < 0.5).float() * 2 - 1
    y = torch.rand((B, 3, 256, 256), generator=g, device="cuda") * 2 - 1
    eager = _trainer("bf16", 16, "normal")
    graphed = _trainer("bf16", 16, "normal")
    replay = graphed.capture(x, m, y, warmup=1)  # 3 eager steps inside
    for _ in range(3):
        eager.train_step(x, m, y)
    assert not _same(_state(eager), _state(graphed))
    for oname in ("optim_G", "optim_D"):  # a different (synthetic) saved state, loaded into both trainers
        sd = copy.deepcopy(getattr(eager, oname).state_dict())
        for st in sd["state"].values():
            st["exp_avg"].mul_(0.5)
            st["exp_avg_sq"].mul_(2.0)
        getattr(eager, oname).load_state_dict(copy.deepcopy(sd))
        getattr(graphed, oname).load_state_dict(copy.deepcopy(sd))
    assert not _same(_state(eager), _state(graphed))
    eager.train_step(x, m, y)
    replay()
    bad = _same(_state(eager), _state(graphed))
    assert not bad, bad[:8]
    # then a replay and an eager (general-path) step of the captured trainer: the step counts carry over
    eager.train_step(x, m, y)
    replay()
    eager.train_step(x, m, y)
    graphed.train_step(x, m, y)
    bad = _same(_state(eager), _state(graphed))
    assert not bad, bad[:8]


def test_splitk_tickets_graph_replay_beside_eager_on_capture_stream():
    """In-launch split-K ticket regions belong to (stream, capture): a graph captured on a stream keeps its own
    region, so its replays (here on another stream) and eager launches on the capture stream's handle never share
    counters.  Both must give the eager result, bit for bit, every time (csrc/igemm_bf16.hip splitk_tickets)."""
    from stcgan_amd import _lib as L
    from stcgan_amd import ops
    BF = torch.bfloat16
    B, Cin, Cout, Hg = 32, 512, 512, 8  # (G's 16 -> 8 conv at bs 32: two in-launch splits)
    _, _, plan = ops.conv_query(L.CONV_S2, B, Hg, Hg, Cin, Cout, BF)
    assert 2 <= plan[2] <= 4, plan
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn((B, 2 * Hg, 2 * Hg, Cin), generator=g, device="cuda").to(BF)
    w = ops.pack(L.PACK_CONV_FWD, torch.randn((Cout, Cin, 4, 4), generator=g, device="cuda") * 0.05, Cout, Cin, BF)
    cap = torch.cuda.Stream()
    other = torch.cuda.Stream()
    ref = torch.empty((B, Hg, Hg, Cout), device="cuda", dtype=BF)
    with torch.cuda.stream(cap):
        pref, _ = ops.conv_stats(L.CONV_S2, B, L.nhwc_view(x), Cin, w, Cout, L.nhwc_view(ref), BF)
    torch.cuda.synchronize()
    yg = torch.empty_like(ref)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=cap):
        pg, _ = ops.conv_stats(L.CONV_S2, B, L.nhwc_view(x), Cin, w, Cout, L.nhwc_view(yg), BF)
    for _ in range(4):
        ye = torch.full_like(ref, float("nan"))
        yg.fill_(float("nan"))
        torch.cuda.synchronize()
        other.wait_stream(torch.cuda.current_stream())
        cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(other):
            graph.replay()
        with torch.cuda.stream(cap):
            pe, _ = ops.conv_stats(L.CONV_S2, B, L.nhwc_view(x), Cin, w, Cout, L.nhwc_view(ye), BF)
        torch.cuda.synchronize()
        assert torch.equal(ye, ref) and torch.equal(yg, ref)
        assert torch.equal(pe, pref) and torch.equal(pg, pref)
