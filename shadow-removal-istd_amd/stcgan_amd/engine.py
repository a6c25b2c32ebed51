"""Whole-network forward/backward orchestration over the HIP kernels.

Each network call is ONE autograd node (GeneratorFn / DiscriminatorFn): the
forward enqueues the layer kernels in order and keeps the raw (pre-BN) conv
outputs plus per-channel BN tables; the backward is written out by hand
(reverse layer order) so that BN-apply/activation work is fused into the GEMM
load prologues and BN backward is fused with the activation backward of every
consumer.  Nothing here computes on the CPU.

Generator layout (STCGAN/networks.py:79-143, pad/crop of
src/models/stcgan_g.py:120-132), with L = num_downs levels, co[k] = conv_k
output channels and S[k] the block-k input resolution
(S[1] = S[0]//2, S[k+1] = ceil(S[k]/2)):
  cat[k] (NHWC, res S[k+1], allocated at the padded size 2*S[k+2]) holds
         [ r_k = conv_k raw output | q_{k+1} = convT_{k+1} raw output ]
  conv_{k+1} reads cat[k][:co_k] with prologue LReLU(BN_k_down(.))  (the in-place
         LeakyReLU of networks.py:106 -- the skip half IS this activation)
  convT_k   reads cat[k] with prologue ReLU(BN(.)) per half           (networks.py:108,143)
  y = tanh(convT_0(ReLU(cat[0])) + bias), written NCHW fp32.
"""
import torch

from . import _lib as L
from . import ops
from .ops import LRELU

# ----------------------------------------------------------------------------- helpers


def _nhwc(B, H, W, C, dt, dev, zero=False):
    f = torch.zeros if zero else torch.empty
    return f((B, H, W, C), dtype=dt, device=dev)


def _half(t, c0, C):
    return t[c0:c0 + C]


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
        self.pindex = {id(p): i for i, p in enumerate(self.params)}


def _sizes(H, W, Lv):
    S = [(H, W), (H // 2, W // 2)]
    for _ in range(2, Lv + 1):
        h, w = S[-1]
        S.append(((h + 1) // 2, (w + 1) // 2))
    return S


def _pad2(S, k):
    """Allocated (padded) size of resolution level k: 2 * S[k+1]."""
    return (2 * S[k + 1][0], 2 * S[k + 1][1])


# ----------------------------------------------------------------------------- generator


def gen_forward(plan, sources, train, dt, cache, save):
    net = plan.net
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

    cat = []
    for k in range(Lv):
        if k < Lv - 1:
            ah, aw = _pad2(S, k + 1)
            cat.append(_nhwc(B, ah, aw, 2 * co[k], dt, dev))
        else:
            cat.append(_nhwc(B, S[Lv][0], S[Lv][1], co[k], dt, dev))
    # prologue tables tab[k] = [scale(2co_k); shift(2co_k)]; level 0 first half is identity (r_0 has no BN)
    tab = [torch.empty((2, 2 * co[k]), dtype=torch.float32, device=dev) for k in range(Lv - 1)]
    tab[0][0, :co[0]].fill_(1.0)
    tab[0][1, :co[0]].zero_()
    st_d, st_u = {}, {}

    def bn_table(bn, xv, C, scale, shift):
        if train:
            return ops.bn_train_table(B, xv, C, dt, bn, scale, shift)
        ops.bn_eval_table(C, bn, scale, shift)
        return None

    # ---- down path
    w0 = ops.packed(cache, plan.conv[0].weight, L.PACK_CONV_FWD, co[0], cin_pad, dt)
    ops.conv(L.CONV_S2, B, L.nhwc_view(xin), cin_pad, w0, co[0], L.nhwc_view(cat[0], 0, *S[1]), dt)
    for k in range(1, Lv):
        wk = ops.packed(cache, plan.conv[k].weight, L.PACK_CONV_FWD, co[k], co[k - 1], dt)
        pro = None if k == 1 else (tab[k - 1][0, :co[k - 1]], tab[k - 1][1, :co[k - 1]])
        ops.conv(L.CONV_S2, B, L.nhwc_view(cat[k - 1], 0, *S[k]), co[k - 1], wk, co[k],
                 L.nhwc_view(cat[k], 0, *S[k + 1]), dt, pro=pro, slope=LRELU)
        if k <= Lv - 2:
            st_d[k] = bn_table(plan.bnd[k], L.nhwc_view(cat[k], 0, *S[k + 1]), co[k],
                               tab[k][0, :co[k]], tab[k][1, :co[k]])
    # ---- up path
    for k in range(Lv - 1, 0, -1):
        cin_t = co[k] if k == Lv - 1 else 2 * co[k]
        wt = ops.packed(cache, plan.convT[k].weight, L.PACK_CONVT_FWD, co[k - 1], cin_t, dt)
        pro = None if k == Lv - 1 else (tab[k][0], tab[k][1])
        ah, aw = _pad2(S, k)
        ops.conv(L.CONVT_S2, B, L.nhwc_view(cat[k], 0, *S[k + 1]), cin_t, wt, co[k - 1],
                 L.nhwc_view(cat[k - 1], co[k - 1], ah, aw), dt, pro=pro, slope=0.0)
        st_u[k] = bn_table(plan.bnu[k], L.nhwc_view(cat[k - 1], co[k - 1], ah, aw), co[k - 1],
                           tab[k - 1][0, co[k - 1]:], tab[k - 1][1, co[k - 1]:])
    # ---- outermost: tanh(convT_0(ReLU(cat[0])) + bias) -> NCHW fp32
    Ho, Wo = 2 * S[1][0], 2 * S[1][1]
    y = torch.empty((B, plan.out_c, Ho, Wo), dtype=torch.float32, device=dev)
    wt0 = ops.packed(cache, plan.convT[0].weight, L.PACK_CONVT_FWD, plan.out_c, 2 * co[0], dt)
    ops.conv(L.CONVT_S2, B, L.nhwc_view(cat[0], 0, *S[1]), 2 * co[0], wt0, plan.out_c, L.nchw_view(y), dt,
             pro=(tab[0][0], tab[0][1]), slope=0.0, bias=plan.convT[0].bias, tanh=True, out_f32=True)
    saved = None
    if save:
        saved = dict(S=S, xin=xin, cat=cat, tab=tab, st_d=st_d, st_u=st_u, y=y, cin=cin, cin_pad=cin_pad,
                     src_c=[s.shape[1] for s in sources])
    return y, saved


def gen_backward(plan, saved, gy, dt, cache, need_src, need_w):
    """Returns (list of source grads (NCHW fp32 or None), dict param-id -> grad)."""
    S, xin, cat, tab = saved["S"], saved["xin"], saved["cat"], saved["tab"]
    st_d, st_u, y = saved["st_d"], saved["st_u"], saved["y"]
    Lv, co = plan.L, plan.co
    dev = y.device
    B = y.shape[0]
    grads = {}
    gy = gy.contiguous()

    def put(p, g):
        if need_w:
            grads[id(p)] = g

    # ---- tanh + bias
    cp = ops.vec(dt)
    Ho, Wo = y.shape[2], y.shape[3]
    dq = _nhwc(B, Ho, Wo, cp, dt, dev)
    dbias0 = ops.tanh_bias_bwd(y, gy, L.nhwc_view(dq), dt)
    put(plan.convT[0].bias, dbias0)
    # ---- up path backward: convT_k, BN_up
    gcat = [None] * Lv
    for k in range(Lv):
        cin_t = co[k] if k == Lv - 1 else 2 * co[k]
        cout_t = plan.out_c if k == 0 else co[k - 1]
        cg = cp if k == 0 else cout_t
        dq_h, dq_w = dq.shape[1], dq.shape[2]
        # convT_k weight gradient: D = transformed cat[k] (grid S[k+1]), G = dq (stride 2)
        if need_w:
            dpro = None if k == Lv - 1 else (tab[k][0], tab[k][1])
            dW = ops.wgrad(B, 2, L.nhwc_view(cat[k], 0, *S[k + 1]), cin_t, L.nhwc_view(dq, 0, dq_h, dq_w), cg,
                           cout_t, dt, dpro=dpro, dslope=0.0, device=dev)
            put(plan.convT[k].weight, dW)
        # input gradient: conv-s2 of dq with the convT weight -> gcat[k] on grid S[k+1]
        wd = ops.packed(cache, plan.convT[k].weight, L.PACK_CONVT_DGRAD, cin_t, cg, dt)
        if k < Lv - 1:
            ah, aw = _pad2(S, k + 1)
            odd = (ah, aw) != S[k + 1]
            gcat[k] = _nhwc(B, ah, aw, cin_t, dt, dev, zero=odd)
        else:
            gcat[k] = _nhwc(B, S[Lv][0], S[Lv][1], cin_t, dt, dev)
        ops.conv(L.CONV_S2, B, L.nhwc_view(dq, 0, dq_h, dq_w), cg, wd, cin_t, L.nhwc_view(gcat[k], 0, *S[k + 1]), dt)
        if k == Lv - 1:
            break
        # BN_up[k+1] backward over q_{k+1} (second half of cat[k], full padded extent)
        ah, aw = _pad2(S, k + 1)
        C = co[k]
        sc, sh = tab[k][0, C:], tab[k][1, C:]
        mean, rstd = st_u[k + 1]
        dq = _nhwc(B, ah, aw, C, dt, dev)
        dg, db = ops.bn_backward(B, L.nhwc_view(cat[k], C, ah, aw), C, dt, L.nhwc_view(dq),
                                 g1=L.nhwc_view(gcat[k], C, ah, aw), s1=0.0,
                                 bn_state=(sc, sh, mean, rstd, plan.bnu[k + 1].weight))
        put(plan.bnu[k + 1].weight, dg)
        put(plan.bnu[k + 1].bias, db)
    # ---- innermost r_{L-1}: ReLU backward (no BN)
    dr = _nhwc(B, S[Lv][0], S[Lv][1], co[Lv - 1], dt, dev)
    ops.bn_backward(B, L.nhwc_view(cat[Lv - 1]), co[Lv - 1], dt, L.nhwc_view(dr), g1=L.nhwc_view(gcat[Lv - 1]),
                    s1=0.0)
    # ---- down path backward: conv_k, BN_down
    src_grads = None
    for k in range(Lv - 1, -1, -1):
        drv = L.nhwc_view(dr, 0, *S[k + 1])
        if k == 0:
            if need_w:
                put(plan.conv[0].weight, ops.wgrad(B, 2, drv, co[0], L.nhwc_view(xin), saved["cin_pad"],
                                                   saved["cin"], dt, device=dev))
            if need_src:
                wd = ops.packed(cache, plan.conv[0].weight, L.PACK_CONV_DGRAD, saved["cin_pad"], co[0], dt)
                gx = _nhwc(B, 2 * S[1][0], 2 * S[1][1], saved["cin_pad"], dt, dev)
                ops.conv(L.CONVT_S2, B, drv, co[0], wd, saved["cin_pad"], L.nhwc_view(gx), dt)
                H, W = S[0]
                src_grads = []
                for c in saved["src_c"]:
                    src_grads.append(torch.zeros((B, c, H, W), dtype=torch.float32, device=dev))
                ops.scatter(gx, src_grads, saved["src_c"], dt, H, W)
            break
        cprev = co[k - 1]
        gpro = None if k == 1 else (tab[k - 1][0, :cprev], tab[k - 1][1, :cprev])
        if need_w:
            put(plan.conv[k].weight, ops.wgrad(B, 2, drv, co[k], L.nhwc_view(cat[k - 1], 0, *S[k]), cprev, cprev,
                                               dt, gpro=gpro, gslope=LRELU, device=dev))
        wd = ops.packed(cache, plan.conv[k].weight, L.PACK_CONV_DGRAD, cprev, co[k], dt)
        ah, aw = 2 * S[k + 1][0], 2 * S[k + 1][1]
        ga = _nhwc(B, ah, aw, cprev, dt, dev)
        ops.conv(L.CONVT_S2, B, drv, co[k], wd, cprev, L.nhwc_view(ga), dt)
        # r_{k-1}: skip (ReLU) + conv_k input (LReLU), then BN_down[k-1] (absent for k-1 == 0)
        dr = _nhwc(B, S[k][0], S[k][1], cprev, dt, dev)
        xv = L.nhwc_view(cat[k - 1], 0, *S[k])
        g1 = L.nhwc_view(gcat[k - 1], 0, *S[k])
        g2 = L.nhwc_view(ga, 0, *S[k])
        if k - 1 == 0:
            ops.bn_backward(B, xv, cprev, dt, L.nhwc_view(dr), g1=g1, s1=0.0, g2=g2, s2=LRELU)
        else:
            mean, rstd = st_d[k - 1]
            bn = plan.bnd[k - 1]
            dg, db = ops.bn_backward(B, xv, cprev, dt, L.nhwc_view(dr), g1=g1, s1=0.0, g2=g2, s2=LRELU,
                                     bn_state=(tab[k - 1][0, :cprev], tab[k - 1][1, :cprev], mean, rstd, bn.weight))
            put(bn.weight, dg)
            put(bn.bias, db)
    return src_grads, grads


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


def disc_forward(plan, sources, train, dt, cache, save):
    dev = sources[0].device
    B, _, H, W = sources[0].shape
    cin = sum(s.shape[1] for s in sources)
    assert cin == plan.in_c, f"discriminator expects {plan.in_c} input channels, got {cin}"
    cin_pad = ops.pad_channels(cin, dt)
    xin = _nhwc(B, H, W, cin_pad, dt, dev)
    ops.gather(sources, xin, dt)
    n = plan.n
    acts = [xin]
    dims = [(H, W)]
    chans = [cin_pad]
    tabs = [None]  # prologue table for reading acts[i] (None = identity)
    stats = [None]
    out = None
    for i, cv in enumerate(plan.convs):
        s = plan.strides[i]
        h, w = _conv_out(dims[-1][0], s), _conv_out(dims[-1][1], s)
        cout = cv.out_channels
        pro, slope = None, None
        if i >= 1:
            slope = LRELU
            if tabs[i] is not None:
                pro = tabs[i]
        mode = L.PACK_CONV_FWD
        wp = ops.packed(cache, cv.weight, mode, cout, chans[i], dt)
        kind = L.CONV_S2 if s == 2 else L.CONV_S1
        if i == n - 1:
            out = torch.empty((B, cout, h, w), dtype=torch.float32, device=dev)
            ops.conv(kind, B, L.nhwc_view(acts[i], 0, *dims[i]), chans[i], wp, cout, L.nchw_view(out), dt, pro=pro,
                     slope=slope, bias=cv.bias, out_f32=True)
            break
        o = _nhwc(B, h, w, cout, dt, dev)
        ops.conv(kind, B, L.nhwc_view(acts[i], 0, *dims[i]), chans[i], wp, cout, L.nhwc_view(o), dt, pro=pro,
                 slope=slope, bias=cv.bias)
        tab, st = None, None
        if i >= 1:
            bn = plan.bns[i - 1]
            t = torch.empty((2, cout), dtype=torch.float32, device=dev)
            if train:
                st = ops.bn_train_table(B, L.nhwc_view(o), cout, dt, bn, t[0], t[1])
            else:
                ops.bn_eval_table(cout, bn, t[0], t[1])
            tab = (t[0], t[1])
        acts.append(o)
        dims.append((h, w))
        chans.append(cout)
        tabs.append(tab)
        stats.append(st)
    saved = None
    if save:
        saved = dict(acts=acts, dims=dims, chans=chans, tabs=tabs, stats=stats, cin=cin, cin_pad=cin_pad,
                     src_c=[s.shape[1] for s in sources], out_shape=tuple(out.shape))
    return out, saved


def disc_backward(plan, saved, gout, dt, cache, need_src, need_w):
    acts, dims, chans, tabs, stats = saved["acts"], saved["dims"], saved["chans"], saved["tabs"], saved["stats"]
    dev = gout.device
    B = gout.shape[0]
    n = plan.n
    grads = {}
    cp = ops.vec(dt)
    h, w = gout.shape[2], gout.shape[3]
    # gradient of the logits [B,1,h,w] -> NHWC with cp channels (R must be a multiple of 4)
    g = _nhwc(B, h, w, cp, dt, dev)
    ops.gather([gout.contiguous()], g, dt)
    gch = cp
    src_grads = None
    for i in range(n - 1, -1, -1):
        cv = plan.convs[i]
        s = plan.strides[i]
        cout = cv.out_channels
        # g: gradient wrt conv_i output (pre-activation / pre-BN), gch channels (>= cout)
        gv = L.nhwc_view(g, 0, h, w)
        pro = tabs[i] if i >= 1 else None
        slope = LRELU if i >= 1 else None
        if need_w:
            dW = ops.wgrad(B, s, gv, gch, L.nhwc_view(acts[i], 0, *dims[i]), chans[i],
                           saved["cin"] if i == 0 else chans[i], dt, gpro=pro, gslope=slope, device=dev)
            grads[id(cv.weight)] = dW[:cout] if gch != cout else dW
            if cv.bias is not None:
                grads[id(cv.bias)] = ops.chan_sum(B, gv, gch, cout, dt, dev)
        if i == 0:
            if need_src:
                wd = ops.packed(cache, cv.weight, L.PACK_CONV_DGRAD, saved["cin_pad"], gch, dt)
                H, W = dims[0]
                gx = _nhwc(B, 2 * h, 2 * w, saved["cin_pad"], dt, dev)
                ops.conv(L.CONVT_S2, B, gv, gch, wd, saved["cin_pad"], L.nhwc_view(gx), dt)
                src_grads = [torch.zeros((B, c, H, W), dtype=torch.float32, device=dev) for c in saved["src_c"]]
                ops.scatter(gx, src_grads, saved["src_c"], dt, H, W)
            break
        # input gradient of conv_i
        ph, pw = dims[i]
        cin = chans[i]
        ga = _nhwc(B, max(ph, 2 * h) if s == 2 else ph, max(pw, 2 * w) if s == 2 else pw, cin, dt, dev)
        if s == 2:
            wd = ops.packed(cache, cv.weight, L.PACK_CONV_DGRAD, cin, gch, dt)
            ops.conv(L.CONVT_S2, B, gv, gch, wd, cin, L.nhwc_view(ga), dt)
        else:
            wd = ops.packed(cache, cv.weight, L.PACK_CONV_S1_DGRAD, cin, gch, dt)
            ops.conv(L.CONV_S1_DGRAD, B, gv, gch, wd, cin, L.nhwc_view(ga, 0, ph, pw), dt)
        # through LReLU (and BN of layer i-1's output, when present)
        gn = _nhwc(B, ph, pw, cin, dt, dev)
        xv = L.nhwc_view(acts[i], 0, ph, pw)
        gav = L.nhwc_view(ga, 0, ph, pw)
        if tabs[i] is None:
            ops.bn_backward(B, xv, cin, dt, L.nhwc_view(gn), g1=gav, s1=LRELU)
        else:
            mean, rstd = stats[i]
            bn = plan.bns[i - 2]
            dg, db = ops.bn_backward(B, xv, cin, dt, L.nhwc_view(gn), g1=gav, s1=LRELU,
                                     bn_state=(tabs[i][0], tabs[i][1], mean, rstd, bn.weight))
            if need_w:
                grads[id(bn.weight)] = dg
                grads[id(bn.bias)] = db
        g, gch, h, w = gn, cin, ph, pw
    return src_grads, grads


# ----------------------------------------------------------------------------- autograd


class NetFn(torch.autograd.Function):
    """One autograd node per network call.  inputs: (ctrl, *sources, *params)."""

    @staticmethod
    def forward(ctx, ctrl, *tensors):
        plan, kind, train, dt, cache, nsrc = ctrl
        sources = [t.contiguous().float() for t in tensors[:nsrc]]
        save = train and any(ctx.needs_input_grad[1:])
        fwd = gen_forward if kind == "G" else disc_forward
        out, saved = fwd(plan, sources, train, dt, cache, save)
        ctx.ctrl = ctrl
        ctx.saved_net = saved
        return out

    @staticmethod
    def backward(ctx, gout):
        plan, kind, train, dt, cache, nsrc = ctx.ctrl
        saved = ctx.saved_net
        if saved is None:
            raise RuntimeError("stcgan_amd: backward through a network called in eval mode is not supported")
        need = ctx.needs_input_grad[1:]
        need_src = any(need[:nsrc])
        need_w = any(need[nsrc:])
        bwd = gen_backward if kind == "G" else disc_backward
        src_grads, grads = bwd(plan, saved, gout, dt, cache, need_src, need_w)
        ctx.saved_net = None
        out = [None]
        for i in range(nsrc):
            out.append(src_grads[i] if (src_grads is not None and need[i]) else None)
        for j, p in enumerate(plan.params):
            out.append(grads.get(id(p)) if need[nsrc + j] else None)
        return tuple(out)
