"""Whole-network forward/backward orchestration over the HIP kernels.

Each network call is ONE autograd node (NetFn): the forward enqueues the layer
kernels in order; the backward is written out by hand in reverse layer order,
with BatchNorm backward fused with the activation backward of every consumer.
Nothing here computes on the CPU.

Activations are materialised once per element by ``stc_bn_apply`` (BN-apply +
LeakyReLU / ReLU), so every GEMM and weight-gradient kernel stages plain operands:
in an implicit GEMM each input element is re-read by 4-16 taps per N tile, so a
fused load-time transform would be paid 4-16x over.

Generator layout (STCGAN/networks.py:79-143, pad/crop of
src/models/stcgan_g.py:120-132), L = num_downs levels, co[k] = conv_k output
channels, S[k] the block-k input resolution (S[1] = S[0]//2, S[k+1] = ceil(S[k]/2)):
  rd[k]  raw conv_k output r_k                    (res S[k+1])
  ad[k]  LeakyReLU(BN_d(r_k)) -> input of conv_{k+1}
         (the in-place LeakyReLU of networks.py:106 -- also the skip half)
  rq[k]  raw convT_k output q_k                   (res 2*S[k+1] = padded S[k])
  cr[k]  [ ReLU(BN_d(r_k)) | ReLU(BN_u(q_{k+1})) ] -> input of convT_k
         (networks.py:108,143: ReLU of the concat; ReLU(LeakyReLU(v)) = ReLU(v))
  y = tanh(convT_0(cr[0]) + bias), written NCHW fp32.
"""
import torch

from . import _lib as L
from . import ops
from .ops import LRELU

# ----------------------------------------------------------------------------- helpers



# ----------------------------------------------------------------------------- tracing (tests)
# TRACE: None, or a dict that collects, per network call, the forward's saved buffers and the backward's
# per-level gradient tensors (tests/test_gpu_c3_layers.py checks every layer against torch on those).
TRACE = None


def _trace(kind, key, t):
    if TRACE is not None:
        TRACE.setdefault(kind, [{}])[-1][key] = t


def _trace_new(kind):
    if TRACE is not None:
        TRACE.setdefault(kind, []).append({})


# ----------------------------------------------------------------------------- weight-gradient lane
# The weight gradients of a backward hang off its input-gradient chain (each needs that layer's incoming
# gradient and saved input; nothing on the chain needs them), so they run on a side stream per calling
# stream and overlap the rest of the chain -- most of the deep (1x1-8x8) layers' kernels are latency-bound
# small grids.  Joined before the backward returns its gradients.
WGRAD_OVERLAP = True
# interleaved A/B (scripts/train_steps.py --ab): round 2: none 13.74, <= 32x32 13.45, <= 64x64 13.64, all 13.75
# ms/step; round 6 (the D-step backward of each discriminator call right after its forward,
# profiles/r06/wgrad_lane/): <= 32x32 10.57, <= 64x64 10.47, all 10.52 ms/step
WGRAD_OVERLAP_MAX_PIX = 64 * 64
_WG_SIDE = {}
# streams (raw handles) whose backward keeps its weight gradients on the stream itself while a HIP graph
# is being captured: the discriminator lanes (STCGAN.capture).  A weight-gradient side stream forked from a
# lane, itself forked from the capturing stream, made the capture's end fault on this ROCm (round-3 probe:
# scripts/graph_capture_probe.py -- lanes alone and side streams of the main stream alone capture fine).
NO_SIDE_IN_CAPTURE = set()
# True: STCGAN.capture keeps the lanes' weight-gradient side streams too (probe switch only: hipStreamEndCapture
# segfaults on this ROCm with them, also when they first fork from the capturing stream and every fork has its own
# event -- profiles/r05/graph_ab/late/)
SIDE_IN_CAPTURE = False


_set_stream = torch._C._cuda_setStream


def _stream_wait(waiter_h, src_h):
    return L.lib().stc_stream_wait(waiter_h, src_h)

# Events recorded or waited on while a HIP graph is being captured, kept alive until the capture has ended
# (STCGAN.capture sets a list here and drops it after capture_end).  torch's Stream.wait_stream and a fork's local
# event are otherwise destroyed inside the open capture, while capture edges still refer to them: the first suspect
# of the hipStreamEndCapture fault with the lanes' weight-gradient side streams (profiles/r05/graph_ab/late/).
CAPTURE_EVENTS = None


def hold(ev):
    """ev, kept alive until the open capture ends (no-op outside a capture)."""
    if CAPTURE_EVENTS is not None:
        CAPTURE_EVENTS.append(ev)
    return ev


def wait_stream(waiter, src):
    """waiter.wait_stream(src), through one library call (stc_stream_wait: a pooled event that outlives an open
    capture)."""
    L.check(L.lib().stc_stream_wait(waiter.cuda_stream, src.cuda_stream), "stc_stream_wait")


class _WgradLane:
    def __init__(self):
        self.cur = torch.cuda.current_stream() if WGRAD_OVERLAP else None
        self.side = None
        self.last_side = False
        if (self.cur is not None and self.cur.cuda_stream in NO_SIDE_IN_CAPTURE
                and torch.cuda.is_current_stream_capturing()):
            self.cur = None
        if self.cur is not None:
            ent = _WG_SIDE.get(self.cur.cuda_stream)
            if ent is None:
                side = torch.cuda.Stream(self.cur.device)
                ent = _WG_SIDE[self.cur.cuda_stream] = (side, side.cuda_stream, self.cur.cuda_stream)
            self.side, self._side_h, self._cur_h = ent

    def run(self, fn, *reads, pixels=0):
        """fn() on the side stream, after everything queued so far on the calling stream; ``reads``: the
        calling stream's tensors fn reads that may be freed before the backward ends.  Only layers of at
        most WGRAD_OVERLAP_MAX_PIX output pixels per image go to the side (the big ones fill the GPU alone;
        overlapping them measured slower).  (The fork is one library call on raw stream handles (stc_stream_wait, a
        pooled event) and a direct current-stream switch: ``Stream.wait_stream`` creates an event per call and
        ``torch.cuda.stream()`` queries the current stream twice -- together ~15 us of host time per call, 50 calls
        per step.)"""
        if self.side is None or pixels > WGRAD_OVERLAP_MAX_PIX:
            self.last_side = False
            return fn()
        self.last_side = True
        side, cur = self.side, self.cur
        L.check(_stream_wait(self._side_h, self._cur_h), "stc_stream_wait")
        for t in reads:
            t.record_stream(side)
        _set_stream(side.stream_id, side.device_index, side.device_type)
        try:
            return fn()
        finally:
            _set_stream(cur.stream_id, cur.device_index, cur.device_type)

    def join(self):
        if self.side is not None:
            L.check(_stream_wait(self._cur_h, self._side_h), "stc_stream_wait")


class GradWriter:
    """Where one backward writes its network's parameter gradients: the network's flat gradient buffer
    (parallel.FlatGrads; each ``p.grad`` is a view of it), so no gradient is allocated, copied into an
    exchange buffer or accumulated by autograd.  torch's accumulation semantics are kept: a parameter
    whose ``.grad`` is None (the optimiser's zero_grad) gets its view and the kernels write it in place; a
    parameter that already holds a gradient (the discriminator's real and fake calls inside one graph,
    STCGAN/stcgan.py:219-227) gets a scratch result that ``flush`` adds to it (one multi-tensor launch),
    old + new in that order.  With data parallelism the network's BucketExchange is told as each layer's
    gradients are enqueued (``done``), so its buckets are all-reduced while the backward continues."""

    def __init__(self, net):
        from .parallel import exchange_of, flat_grads
        self.flat = flat_grads(net)
        self.exchange = exchange_of(net)
        self.acc = []
        self._acc_ids = set()

    def dest(self, p):
        g = p.grad
        if g is None:
            p.grad = self.flat.view(p)
            return p.grad
        if not self.flat.owns(g, p):
            # a gradient that is not this network's flat-buffer view (assigned by the caller, or carried along by
            # a module move): moved into the view, so that the exchange averages what the optimiser reads
            v = self.flat.view(p)
            v.copy_(g)
            p.grad = g = v
        s = torch.empty(p.shape, dtype=torch.float32, device=p.device)
        self.acc.append((g, s, p))
        self._acc_ids.add(id(p))
        return s

    def done(self, params, lane=None):
        """Gradients of ``params`` enqueued (on the lane's side stream when its last job went there)."""
        if self.exchange is None:
            return
        fresh = [p for p in params if id(p) not in self._acc_ids]
        if fresh:
            side = lane.side if (lane is not None and getattr(lane, "last_side", False)) else None
            self.exchange.ready(fresh, side)

    def flush(self):
        if self.acc:
            ops.grad_accumulate([(g, s) for g, s, _ in self.acc])
            if self.exchange is not None:
                self.exchange.ready([p for _, _, p in self.acc])
            self.acc, self._acc_ids = [], set()


_ONES = {}


def _ones_plane(B, H, W, dev):
    """A persistent [B, 1, H, W] fp32 plane of ones (filled once, synchronously: streams share it)."""
    key = (B, H, W, str(dev))
    t = _ONES.get(key)
    if t is None:
        t = _ONES[key] = torch.ones((B, 1, H, W), dtype=torch.float32, device=dev)
        torch.cuda.current_stream(dev).synchronize()
    return t


def _nhwc(B, H, W, C, dt, dev, zero=False):
    f = torch.zeros if zero else torch.empty
    return f((B, H, W, C), dtype=dt, device=dev)


class GenPlan:
    """Static structure of a UnetGenerator module (parameters by role)."""

    def __init__(self, net):
        self.net = net
        outer = net.model  # outermost UnetSkipConnectionBlock
        self.in_c = outer.model[0].in_channels
        self.out_c = outer.model[3].out_channels
        conv, bnd, convT, bnu = [], {}, {}, {}
        conv.append(outer.model[0])
        convT[0] = outer.model[3]
        blk = outer.model[1]
        k = 1
        while True:
            seq = blk.model
            conv.append(seq[1])
            if blk.innermost:
                convT[k] = seq[3]
                bnu[k] = seq[4]
                break
            bnd[k] = seq[2]
            convT[k] = seq[5]
            bnu[k] = seq[6]
            blk = seq[3]
            k += 1
        self.L = len(conv)
        self.conv, self.bnd, self.convT, self.bnu = conv, bnd, convT, bnu
        self.co = [c.out_channels for c in conv]
        self.params = list(net.parameters())


def _sizes(H, W, Lv):
    S = [(H, W), (H // 2, W // 2)]
    for _ in range(2, Lv + 1):
        h, w = S[-1]
        S.append(((h + 1) // 2, (w + 1) // 2))
    return S


def _pad2(S, k):
    """Padded size of resolution level k: 2 * S[k+1] (the extent a ConvT from level k+1 produces)."""
    return (2 * S[k + 1][0], 2 * S[k + 1][1])


def _conv_bn(kind, B, xv, cin, w, cout, yv, dt, bn, train, dev):
    """Conv whose output feeds a BatchNorm2d: returns ((2, cout) scale/shift table, (mean, rstd) or None).
    Train mode: the batch statistics come out of the conv itself (stc_conv_fwd_ex)."""
    t = torch.empty((2, cout), dtype=torch.float32, device=dev)
    if train:
        part, nch = ops.conv_stats(kind, B, xv, cin, w, cout, yv, dt)
        st = ops.bn_finalize_part(part, nch, cout, bn, t[0], t[1])
    else:
        ops.conv(kind, B, xv, cin, w, cout, yv, dt)
        ops.bn_eval_table(cout, bn, t[0], t[1])
        st = None
    return t, st


def _conv_bn_act(kind, B, xv, cin, w, cout, yv, dt, bn, train, dev, apply_x, y1, s1, y2=None, s2=0.0, defer=None):
    """Conv -> BatchNorm2d -> activation pass of ``apply_x`` into y1 [and y2] (y1 None: none); returns _conv_bn's
    (table, (mean, rstd) or None).  Train mode: one library call (ops.conv_bn_act); ``defer`` (a list): the running
    statistics are not updated, the update's inputs are appended (ops.bn_running_update)."""
    if train:
        return ops.conv_bn_act(kind, B, xv, cin, w, cout, yv, dt, bn, apply_x, y1, s1, y2, s2, defer=defer)
    t, st = _conv_bn(kind, B, xv, cin, w, cout, yv, dt, bn, train, dev)
    if y1 is not None:
        ops.bn_apply(B, apply_x, cout, dt, (t[0], t[1]), y1, s1, y2, s2)
    return t, st


# ----------------------------------------------------------------------------- generator


def gen_forward(plan, sources, train, dt, cache, save):
    dev = sources[0].device
    B, _, H, W = sources[0].shape
    Lv, co = plan.L, plan.co
    S = _sizes(H, W, Lv)
    assert S[Lv][0] >= 1 and S[Lv][1] >= 1, "input too small for the generator depth"
    cin = sum(s.shape[1] for s in sources)
    assert cin == plan.in_c, f"generator expects {plan.in_c} input channels, got {cin}"
    cin_pad = ops.pad_channels(cin, dt)
    xin = _nhwc(B, H, W, cin_pad, dt, dev)
    ops.gather(sources, xin, dt)

    def cin_t(k):
        return co[k] if k == Lv - 1 else 2 * co[k]

    rd = [None] + [_nhwc(B, *S[k + 1], co[k], dt, dev) for k in range(1, Lv)]  # (rd[0]: below)
    ad = [_nhwc(B, *S[k + 1], co[k], dt, dev) if k < Lv - 1 else None for k in range(Lv)]
    cr = [_nhwc(B, *S[k + 1], cin_t(k), dt, dev) for k in range(Lv)]
    rq = [None] + [_nhwc(B, *_pad2(S, k), co[k - 1], dt, dev) for k in range(1, Lv)]
    tab_d, tab_u, st_d, st_u = {}, {}, {}, {}

    def conv_bn_act(kind, xv, cin_, w, cout, yv, bn, apply_x, y1, s1, y2=None, s2=0.0):
        """conv -> BatchNorm (batch statistics fused into the conv in train mode) -> activation pass."""
        return _conv_bn_act(kind, B, xv, cin_, w, cout, yv, dt, bn, train, dev, apply_x, y1, s1, y2, s2)

    # ---- down path
    w0 = ops.packed(cache, plan.conv[0].weight, L.PACK_CONV_FWD, co[0], cin_pad, dt)
    if ops.conv_act(L.CONV_S2, B, L.nhwc_view(xin), cin_pad, w0, co[0], L.nhwc_view(ad[0]), LRELU, dt,
                    L.nhwc_view(cr[0], 0), 0.0):
        # no raw r_0: its only reader, the backward's ReLU/LeakyReLU test, sees the same signs in ad[0]
        rd[0] = ad[0]
    else:
        rd[0] = _nhwc(B, *S[1], co[0], dt, dev)
        ops.conv(L.CONV_S2, B, L.nhwc_view(xin), cin_pad, w0, co[0], L.nhwc_view(rd[0]), dt)
        ops.bn_apply(B, L.nhwc_view(rd[0]), co[0], dt, None, L.nhwc_view(ad[0]), LRELU,
                     L.nhwc_view(cr[0], 0), 0.0)
    for k in range(1, Lv):
        wk = ops.packed(cache, plan.conv[k].weight, L.PACK_CONV_FWD, co[k], co[k - 1], dt)
        if k <= Lv - 2:
            rv = L.nhwc_view(rd[k])
            tab_d[k], st_d[k] = conv_bn_act(L.CONV_S2, L.nhwc_view(ad[k - 1]), co[k - 1], wk, co[k], rv, plan.bnd[k],
                                            rv, L.nhwc_view(ad[k]), LRELU, L.nhwc_view(cr[k], 0), 0.0)
        else:  # innermost: no down-norm (STCGAN/networks.py:118-124)
            ops.conv(L.CONV_S2, B, L.nhwc_view(ad[k - 1]), co[k - 1], wk, co[k], L.nhwc_view(rd[k]), dt)
            ops.bn_apply(B, L.nhwc_view(rd[k]), co[k], dt, None, L.nhwc_view(cr[k]), 0.0)
    # ---- up path
    for k in range(Lv - 1, 0, -1):
        wt = ops.packed(cache, plan.convT[k].weight, L.PACK_CONVT_FWD, co[k - 1], cin_t(k), dt)
        # statistics over the full ConvT extent (before the crop of an odd level)
        tab_u[k], st_u[k] = conv_bn_act(L.CONVT_S2, L.nhwc_view(cr[k]), cin_t(k), wt, co[k - 1], L.nhwc_view(rq[k]),
                                        plan.bnu[k], L.nhwc_view(rq[k], 0, *S[k]), L.nhwc_view(cr[k - 1], co[k - 1]),
                                        0.0)
    # ---- outermost: tanh(convT_0(cr[0]) + bias) -> NCHW fp32
    Ho, Wo = 2 * S[1][0], 2 * S[1][1]
    y = torch.empty((B, plan.out_c, Ho, Wo), dtype=torch.float32, device=dev)
    wt0 = ops.packed(cache, plan.convT[0].weight, L.PACK_CONVT_FWD, plan.out_c, 2 * co[0], dt)
    ops.conv(L.CONVT_S2, B, L.nhwc_view(cr[0]), 2 * co[0], wt0, plan.out_c, L.nchw_view(y), dt,
             bias=plan.convT[0].bias, tanh=True, out_f32=True)
    saved = None
    if save:
        saved = dict(S=S, xin=xin, rd=rd, ad=ad, cr=cr, rq=rq, tab_d=tab_d, tab_u=tab_u, st_d=st_d, st_u=st_u,
                     y=y, cin=cin, cin_pad=cin_pad, src_c=[s.shape[1] for s in sources])
        if TRACE is not None:
            _trace_new("G")
            _trace("G", "saved", saved)
    return y, saved


def gen_backward(plan, saved, gy, dt, cache, need_src, W):
    """Returns the list of source grads (NCHW fp32 or None); the parameter gradients go to the
    GradWriter ``W`` (None: not needed)."""
    S, xin, rd, ad, cr, rq = saved["S"], saved["xin"], saved["rd"], saved["ad"], saved["cr"], saved["rq"]
    tab_d, tab_u, st_d, st_u, y = saved["tab_d"], saved["tab_u"], saved["st_d"], saved["st_u"], saved["y"]
    Lv, co = plan.L, plan.co
    dev = y.device
    B = y.shape[0]
    gy = gy.contiguous()
    need_w = W is not None
    lane = _WgradLane() if need_w else None

    def dest(p):
        return W.dest(p) if need_w else None

    # ---- tanh + bias
    cp = ops.vec(dt)
    Ho, Wo = y.shape[2], y.shape[3]
    dq = _nhwc(B, Ho, Wo, cp, dt, dev)
    ops.tanh_bias_bwd(y, gy, L.nhwc_view(dq), dt, dbias=dest(plan.convT[0].bias))
    if need_w:
        W.done([plan.convT[0].bias])
    _trace("G", ("dq", 0), dq)
    # ---- up path backward: convT_k, then BN_up[k+1]
    gcat = [None] * Lv
    for k in range(Lv):
        cin_t = co[k] if k == Lv - 1 else 2 * co[k]
        cout_t = plan.out_c if k == 0 else co[k - 1]
        cg = cp if k == 0 else cout_t
        dqv = L.nhwc_view(dq)
        if need_w:  # D = convT input (grid S[k+1]), G = dq gathered at stride 2
            wT = plan.convT[k].weight
            lane.run(lambda k=k, dqv=dqv, cin_t=cin_t, cg=cg, cout_t=cout_t, out=W.dest(wT): ops.wgrad(
                B, 2, L.nhwc_view(cr[k]), cin_t, dqv, cg, cout_t, dt, device=dev, out=out), dq,
                pixels=S[k + 1][0] * S[k + 1][1])
        wd = ops.packed(cache, plan.convT[k].weight, L.PACK_CONVT_DGRAD, cin_t, cg, dt)
        if k < Lv - 1:
            ah, aw = _pad2(S, k + 1)
            gcat[k] = _nhwc(B, ah, aw, cin_t, dt, dev, zero=(ah, aw) != S[k + 1])
        else:
            gcat[k] = _nhwc(B, *S[Lv], cin_t, dt, dev)
        _trace("G", ("gcat", k), gcat[k])
        if k == Lv - 1:
            ops.conv(L.CONV_S2, B, dqv, cg, wd, cin_t, L.nhwc_view(gcat[k], 0, *S[k + 1]), dt)
            if need_w:  # (after the last read of the weight: the optimiser may update it from here on)
                W.done([plan.convT[k].weight], lane)
            break
        # BN_up[k+1] over q_{k+1}: full (padded) extent; the cropped rows carry zero gradient.
        # Its gradient is the second half of gcat[k] (ReLU of the concat), so the BN reduction
        # is fused into the conv that writes gcat[k] (channels C..2C -> BN channels 0..C).
        ah, aw = _pad2(S, k + 1)
        C = co[k]
        mean, rstd = st_u[k + 1]
        t = tab_u[k + 1]
        dq = _nhwc(B, ah, aw, C, dt, dev)
        bn = plan.bnu[k + 1]
        ops.conv_bn_backward(L.CONV_S2, B, dqv, cg, wd, cin_t, L.nhwc_view(gcat[k], 0, *S[k + 1]), dt,
                             bn_x=L.nhwc_view(rq[k + 1]), C=C, bn_state=(t[0], t[1], mean, rstd),
                             gamma=bn.weight, s_self=0.0, ch_off=C, dxv=L.nhwc_view(dq),
                             dgamma=dest(bn.weight), dbeta=dest(bn.bias))
        if need_w:
            W.done([plan.convT[k].weight], lane)
            W.done([bn.weight, bn.bias])
        _trace("G", ("dq", k + 1), dq)
    # ---- innermost r_{L-1}: ReLU backward (no BN)
    dr = _nhwc(B, *S[Lv], co[Lv - 1], dt, dev)
    ops.bn_backward(B, L.nhwc_view(rd[Lv - 1]), co[Lv - 1], dt, L.nhwc_view(dr), g1=L.nhwc_view(gcat[Lv - 1]),
                    s1=0.0)
    # ---- down path backward: conv_k, then BN_down[k-1]
    src_grads = None
    for k in range(Lv - 1, -1, -1):
        drv = L.nhwc_view(dr)
        _trace("G", ("dr", k), dr)
        if k == 0:
            if need_w:
                w0 = plan.conv[0].weight
                lane.run(lambda drv=drv, out=W.dest(w0): ops.wgrad(
                    B, 2, drv, co[0], L.nhwc_view(xin), saved["cin_pad"], saved["cin"], dt, device=dev, out=out),
                    dr, pixels=S[1][0] * S[1][1])
            if need_src:
                wd = ops.packed(cache, plan.conv[0].weight, L.PACK_CONV_DGRAD, saved["cin_pad"], co[0], dt)
                gx = _nhwc(B, 2 * S[1][0], 2 * S[1][1], saved["cin_pad"], dt, dev)
                ops.conv(L.CONVT_S2, B, drv, co[0], wd, saved["cin_pad"], L.nhwc_view(gx), dt)
                H, W_ = S[0]
                # only the sources that need a gradient; the scatter writes every element of those
                src_grads = [torch.empty((B, c, H, W_), dtype=torch.float32, device=dev) if nd else None
                             for c, nd in zip(saved["src_c"], need_src)]
                ops.scatter(gx, src_grads, saved["src_c"], dt, H, W_)
            if need_w:
                W.done([plan.conv[0].weight], lane)
            break
        cprev = co[k - 1]
        if need_w:  # D = dr_k (grid S[k+1]), G = conv_k input = ad[k-1]
            wk = plan.conv[k].weight
            lane.run(lambda k=k, drv=drv, cprev=cprev, out=W.dest(wk): ops.wgrad(
                B, 2, drv, co[k], L.nhwc_view(ad[k - 1]), cprev, cprev, dt, device=dev, out=out), dr,
                pixels=S[k + 1][0] * S[k + 1][1])
        wd = ops.packed(cache, plan.conv[k].weight, L.PACK_CONV_DGRAD, cprev, co[k], dt)
        ga = _nhwc(B, 2 * S[k + 1][0], 2 * S[k + 1][1], cprev, dt, dev)
        _trace("G", ("ga", k), ga)
        # r_{k-1} feeds the skip (ReLU) and conv_k (LeakyReLU); then BN_down[k-1] (absent for k-1 == 0)
        dr = _nhwc(B, *S[k], cprev, dt, dev)
        xv = L.nhwc_view(rd[k - 1])
        g1 = L.nhwc_view(gcat[k - 1], 0, *S[k])
        if k - 1 == 0:
            # r_0 has no BatchNorm: the activation backward (LeakyReLU into conv_1, ReLU into the skip) in the
            # input-gradient conv's epilogue when it has one (no ga tensor), else conv + bn_backward
            if TRACE is not None or (ga.shape[1], ga.shape[2]) != tuple(S[k]) or not ops.conv_act_backward(
                    L.CONVT_S2, B, drv, co[k], wd, cprev, L.nhwc_view(dr), dt, act_x=xv, s_self=LRELU, g_other=g1,
                    s_other=0.0):
                ops.conv(L.CONVT_S2, B, drv, co[k], wd, cprev, L.nhwc_view(ga), dt)
                ops.bn_backward(B, xv, cprev, dt, L.nhwc_view(dr), g1=g1, s1=0.0, g2=L.nhwc_view(ga, 0, *S[k]),
                                s2=LRELU)
            if need_w:
                W.done([plan.conv[k].weight], lane)
        else:  # BN reduction fused into the input-gradient conv that produces ga
            mean, rstd = st_d[k - 1]
            t = tab_d[k - 1]
            bn = plan.bnd[k - 1]
            ops.conv_bn_backward(L.CONVT_S2, B, drv, co[k], wd, cprev, L.nhwc_view(ga), dt, bn_x=xv, C=cprev,
                                 bn_state=(t[0], t[1], mean, rstd), gamma=bn.weight, s_self=LRELU,
                                 g_other=g1, s_other=0.0, dxv=L.nhwc_view(dr), dgamma=dest(bn.weight),
                                 dbeta=dest(bn.bias))
            if need_w:
                W.done([plan.conv[k].weight], lane)
                W.done([bn.weight, bn.bias])
    if lane is not None:
        lane.join()
    return src_grads


# ----------------------------------------------------------------------------- discriminator


class DiscPlan:
    """NLayerDiscriminator (STCGAN/networks.py:147-192): conv+bias, LReLU, [conv, BN, LReLU] x n, conv+bias."""

    def __init__(self, net):
        self.net = net
        seq = net.model
        convs = [m for m in seq if isinstance(m, torch.nn.Conv2d)]
        bns = [m for m in seq if isinstance(m, torch.nn.BatchNorm2d)]
        assert len(convs) == len(bns) + 2
        self.convs, self.bns = convs, bns
        self.n = len(convs)
        self.strides = [c.stride[0] for c in convs]
        self.in_c = convs[0].in_channels
        self.params = list(net.parameters())


def _conv_out(h, s):
    return (h + 2 - 4) // s + 1


def disc_forward(plan, sources, train, dt, cache, save, inputs=None, stats_only=False, defer=None):
    """raw[i] = conv_{i-1} raw output (raw[0] = padded input); act[i] = input of conv_i.
    inputs: optional dict reusing the gathered NHWC input across calls on the same source tensors
    (the trainer's real/fake pairs are fed to each discriminator twice per step, STCGAN/stcgan.py:215-280;
    valid while those tensors are alive and unmodified -- one train step)."""
    dev = sources[0].device
    B, _, H, W = sources[0].shape
    cin = sum(s.shape[1] for s in sources)
    assert cin == plan.in_c, f"discriminator expects {plan.in_c} input channels, got {cin}"
    cin_pad = ops.pad_channels(cin, dt)
    # first-layer bias gradient for free: a constant-1 plane in the first padding channel (its packed weights
    # are zero) makes the weight gradient's tap (1,1) of that channel sum the output gradient over every pixel
    # (k4 s2 p1: input row 2*o + kh - 1 = 2*o is always inside), replacing a full pass over that gradient
    bias_ch = cin if (plan.convs[0].bias is not None and cin < cin_pad and len(sources) < 4
                      and plan.strides[0] == 2) else None
    key = None
    if inputs is not None:
        key = tuple((s.data_ptr(), s._version, tuple(s.shape)) for s in sources) + (dt, cin_pad)
    xin = inputs.get(key) if key is not None else None
    if xin is None:
        xin = _nhwc(B, H, W, cin_pad, dt, dev)
        ops.gather(list(sources) + ([_ones_plane(B, H, W, dev)] if bias_ch is not None else []), xin, dt)
        if key is not None:
            inputs[key] = xin
    n = plan.n
    raw, act, dims, chans, tabs, stats = [xin], [xin], [(H, W)], [cin_pad], [None], [None]
    out = None
    for i, cv in enumerate(plan.convs):
        s = plan.strides[i]
        if s == 2:
            assert dims[i][0] % 2 == 0 and dims[i][1] % 2 == 0, "stride-2 discriminator layers need even sizes"
        h, w = _conv_out(dims[i][0], s), _conv_out(dims[i][1], s)
        cout = cv.out_channels
        wp = ops.packed(cache, cv.weight, L.PACK_CONV_FWD, cout, chans[i], dt)
        kind = L.CONV_S2 if s == 2 else L.CONV_S1
        if i == n - 1:
            if stats_only:  # logits not computed: a zero-element placeholder, so that no caller can read garbage
                out = torch.empty((B, cout, 0, 0), dtype=torch.float32, device=dev)
                break
            out = torch.empty((B, cout, h, w), dtype=torch.float32, device=dev)
            ops.conv(kind, B, L.nhwc_view(act[i]), chans[i], wp, cout, L.nchw_view(out), dt, bias=cv.bias,
                     out_f32=True)
            break
        tab, st = None, None
        a = _nhwc(B, h, w, cout, dt, dev)
        if i >= 1:  # conv -> BatchNorm -> LeakyReLU (networks.py:167-180); no conv bias there
            assert cv.bias is None
            o = _nhwc(B, h, w, cout, dt, dev)
            ov = L.nhwc_view(o)
            # (stats_only: only the logits layer reads the last activation -- no pass)
            t, st = _conv_bn_act(kind, B, L.nhwc_view(act[i]), chans[i], wp, cout, ov, dt, plan.bns[i - 1], train,
                                 dev, ov, None if (stats_only and i == n - 2) else L.nhwc_view(a), LRELU, defer=defer)
            tab = (t[0], t[1])
        elif ops.conv_act(kind, B, L.nhwc_view(act[i]), chans[i], wp, cout, L.nhwc_view(a), LRELU, dt, bias=cv.bias):
            o = a  # no raw output: the backward's LeakyReLU test sees the same signs in the activation
        else:
            o = _nhwc(B, h, w, cout, dt, dev)
            ops.conv(kind, B, L.nhwc_view(act[i]), chans[i], wp, cout, L.nhwc_view(o), dt, bias=cv.bias)
            ops.bn_apply(B, L.nhwc_view(o), cout, dt, tab, L.nhwc_view(a), LRELU)
        raw.append(o)
        act.append(a)
        dims.append((h, w))
        chans.append(cout)
        tabs.append(tab)
        stats.append(st)
    saved = None
    if save:
        saved = dict(raw=raw, act=act, dims=dims, chans=chans, tabs=tabs, stats=stats, cin=cin, cin_pad=cin_pad,
                     bias_ch=bias_ch,
                     src_c=[s.shape[1] for s in sources])
        if TRACE is not None:
            _trace_new("D")
            _trace("D", "saved", saved)
    return out, saved


def disc_backward(plan, saved, gout, dt, cache, need_src, W):
    """Returns the list of source grads (NCHW fp32 or None); parameter gradients go to the GradWriter ``W``."""
    raw, act, dims, chans, tabs, stats = (saved["raw"], saved["act"], saved["dims"], saved["chans"], saved["tabs"],
                                          saved["stats"])
    dev = gout.device
    B = gout.shape[0]
    n = plan.n
    need_w = W is not None
    cp = ops.vec(dt)
    h, w = gout.shape[2], gout.shape[3]
    # gradient of the logits [B,1,h,w] -> NHWC with cp channels (channel counts are vector multiples)
    g = _nhwc(B, h, w, cp, dt, dev)
    ops.gather([gout.contiguous()], g, dt)
    gch = cp
    src_grads = None
    lane = _WgradLane() if need_w else None
    for i in range(n - 1, -1, -1):
        cv = plan.convs[i]
        s = plan.strides[i]
        cout = cv.out_channels
        gv = L.nhwc_view(g, 0, h, w)  # gradient wrt conv_i output (pre-activation / pre-BN), gch channels
        _trace("D", ("g", i), g)
        if need_w:
            bc = saved["bias_ch"] if i == 0 else None
            if bc is None:
                dw_out = W.dest(cv.weight)
                db_out = W.dest(cv.bias) if cv.bias is not None else None
            else:  # the weight gradient of the padded input (+ the constant-1 channel) goes through a scratch
                dw_out, db_out = W.dest(cv.weight), W.dest(cv.bias)

            def wg(i=i, s=s, cout=cout, gv=gv, gch=gch, cv=cv, bc=bc, dw_out=dw_out, db_out=db_out):
                if bc is not None:  # the constant-1 channel's tap (1,1) is the bias gradient (disc_forward)
                    dW = ops.wgrad(B, s, gv, gch, L.nhwc_view(act[i]), chans[i], bc + 1, dt, device=dev, rows=cout)
                    dw_out.copy_(dW[:cout, :saved["cin"]])
                    db_out.copy_(dW[:cout, bc, 1, 1])
                    return
                ops.wgrad(B, s, gv, gch, L.nhwc_view(act[i]), chans[i], saved["cin"] if i == 0 else chans[i], dt,
                          device=dev, rows=cout, out=dw_out)
                if cv.bias is not None:
                    ops.chan_sum(B, gv, gch, cout, dt, dev, out=db_out)
            lane.run(wg, g, pixels=h * w)
        own = [cv.weight] + ([cv.bias] if cv.bias is not None else [])
        if i == 0:
            if need_src:
                wd = ops.packed(cache, cv.weight, L.PACK_CONV_DGRAD, saved["cin_pad"], gch, dt)
                H, W_ = dims[0]
                gx = _nhwc(B, 2 * h, 2 * w, saved["cin_pad"], dt, dev)
                ops.conv(L.CONVT_S2, B, gv, gch, wd, saved["cin_pad"], L.nhwc_view(gx), dt)
                # only the sources that need a gradient; the scatter writes every element of those
                src_grads = [torch.empty((B, c, H, W_), dtype=torch.float32, device=dev) if nd else None
                             for c, nd in zip(saved["src_c"], need_src)]
                ops.scatter(gx, src_grads, saved["src_c"], dt, H, W_)
            if need_w:
                W.done(own, lane)
            break
        # input gradient of conv_i (grad wrt act[i])
        ph, pw = dims[i]
        cin = chans[i]
        ga = _nhwc(B, ph, pw, cin, dt, dev)
        if s == 2:
            wd = ops.packed(cache, cv.weight, L.PACK_CONV_DGRAD, cin, gch, dt)
            dkind = L.CONVT_S2
        else:
            wd = ops.packed(cache, cv.weight, L.PACK_CONV_S1_DGRAD, cin, gch, dt)
            dkind = L.CONV_S1_DGRAD
        # through LeakyReLU (and the BN of layer i-1's output, when present: its reduction fused
        # into the input-gradient conv)
        gn = _nhwc(B, ph, pw, cin, dt, dev)
        _trace("D", ("ga", i), ga)
        xv = L.nhwc_view(raw[i])
        if tabs[i] is None:  # (no BatchNorm: the LeakyReLU backward in the conv epilogue when it has one)
            if TRACE is not None or not ops.conv_act_backward(dkind, B, gv, gch, wd, cin, L.nhwc_view(gn), dt, act_x=xv,
                                                              s_self=LRELU):
                ops.conv(dkind, B, gv, gch, wd, cin, L.nhwc_view(ga), dt)
                ops.bn_backward(B, xv, cin, dt, L.nhwc_view(gn), g1=L.nhwc_view(ga), s1=LRELU)
            if need_w:
                W.done(own, lane)
        else:
            mean, rstd = stats[i]
            bn = plan.bns[i - 2]
            ops.conv_bn_backward(dkind, B, gv, gch, wd, cin, L.nhwc_view(ga), dt, bn_x=xv, C=cin,
                                 bn_state=(tabs[i][0], tabs[i][1], mean, rstd), gamma=bn.weight,
                                 s_self=LRELU, dxv=L.nhwc_view(gn),
                                 dgamma=W.dest(bn.weight) if need_w else None,
                                 dbeta=W.dest(bn.bias) if need_w else None)
            if need_w:
                W.done(own, lane)
                W.done([bn.weight, bn.bias])
        g, gch, h, w = gn, cin, ph, pw
    if lane is not None:
        lane.join()
    return src_grads


# ----------------------------------------------------------------------------- autograd


class NetFn(torch.autograd.Function):
    """One autograd node per network call.  inputs: (ctrl, *sources, *params).

    The backward returns gradients for the sources only: the parameters' gradients are written by the
    kernels straight into the network's flat gradient buffer (GradWriter), so autograd never allocates,
    accumulates or hooks them (``p.grad`` is set by the backward itself)."""

    @staticmethod
    def forward(ctx, ctrl, *tensors):
        plan, kind, train, dt, cache, nsrc, inputs, _, stats_only, defer = ctrl
        sources = [t.contiguous().float() for t in tensors[:nsrc]]
        save = train and any(ctx.needs_input_grad[1:])
        ops.refresh_packs(cache)  # all operands packed since the last optimiser step, one launch
        out, saved = (gen_forward(plan, sources, train, dt, cache, save) if kind == "G" else
                      disc_forward(plan, sources, train, dt, cache, save, inputs, stats_only and not save, defer))
        ctx.ctrl = ctrl
        ctx.saved_net = saved
        return out

    @staticmethod
    def backward(ctx, gout):
        plan, kind, train, dt, cache, nsrc, _, consumer, _, _ = ctx.ctrl
        saved = ctx.saved_net
        if saved is None:
            raise RuntimeError("stcgan_amd: backward through a network called in eval mode is not supported")
        need = ctx.needs_input_grad[1:]
        need_src = list(need[:nsrc]) if any(need[:nsrc]) else None  # per source, or None
        W = GradWriter(plan.net) if any(need[nsrc:]) else None
        if gout.is_cuda:
            # a side-stream network's incoming gradient is allocated on the main stream (the loss
            # backward): autograd orders this stream after it, but does not keep the caching allocator
            # from handing the block back to the main stream once this Python call returns, while the
            # kernels enqueued here may still read it
            gout.record_stream(torch.cuda.current_stream(gout.device))
        bwd = gen_backward if kind == "G" else disc_backward
        src_grads = bwd(plan, saved, gout, dt, cache, need_src, W)
        if W is not None:
            W.flush()
        ctx.saved_net = None
        out = [None]
        for i in range(nsrc):
            out.append(src_grads[i] if (src_grads is not None and need[i]) else None)
            if consumer is not None and out[-1] is not None:
                # a side-stream network's input gradient is read (and freed) on the consumer's stream: keep
                # its block from being reused on this stream before the consumer is done with it
                out[-1].record_stream(consumer)
        out.extend([None] * len(plan.params))
        return tuple(out)
