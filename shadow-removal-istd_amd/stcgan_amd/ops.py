"""Thin tensor-level wrappers over the C-ABI (include/stcgan_hip.h).

Every function here enqueues HIP kernels of libstcgan_hip.so on torch's current
stream; torch is used only for device memory (caching allocator) and streams.
"""
import ctypes

import torch

from . import _lib as L
from ._lib import check, lib, ptr, stream

LRELU = 0.2
BN_EPS = 1e-5
BN_MOMENTUM = 0.1


def vec(dt):
    """Elements per 16-byte chunk for the activation dtype."""
    return 4 if dt == torch.float32 else 8


def pad_channels(c, dt):
    """Smallest power of two >= max(c, vec(dt))."""
    p = vec(dt)
    while p < c:
        p *= 2
    return p


def _ws(nbytes, device):
    if nbytes <= 0:
        return None, 0
    return torch.empty(int(nbytes), dtype=torch.uint8, device=device), int(nbytes)


def _pro(pro):
    if pro is None:
        return None, None
    sc, sh = pro
    return ptr(sc), ptr(sh)


# Instrumentation (bench.py / scripts): when a list, conv()/conv_stats()/conv_bn_backward()/wgrad() append
# (kernel, single-kernel call, flops, start event, end event, description); the events bracket the call's
# MAIN kernel only (stc_time_next_main_kernel), not a split-K / split-pixel reduction it enqueues after it.
_timer = None
# when a list: wgrad() also appends (kernel, start, end) events around the WHOLE call (main kernel + its
# split-pixel reduction), so that the roofline can charge the reduction to the kernel
_call_timer = None


def _main_events():
    """A pair of timing events armed to bracket the next main kernel this thread launches."""
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()  # creates the events; the library records them again around the kernel
    e1.record()
    check(lib().stc_time_next_main_kernel(ctypes.c_void_p(e0.cuda_event), ctypes.c_void_p(e1.cuda_event)),
          "stc_time_next_main_kernel")
    return e0, e1


def _disarm():
    lib().stc_time_next_main_kernel(None, None)


# Plan / workspace answers of the library are pure functions of their arguments (no environment, no device
# state), and the step asks the same few dozen questions every iteration: memoised, ~5 us of host time per call.
_MEMO = {}


def _conv_ws_bytes(kind, B, gh, gw, cin, cout, dt):
    key = ("cws", kind, B, gh, gw, cin, cout, dt)
    v = _MEMO.get(key)
    if v is None:
        v = _MEMO[key] = lib().stc_conv_fwd_workspace(L.dtype_code(dt), kind, B, gh, gw, cin, cout)
    return v


def set_splitk_inlaunch(on):
    """Split-K combined inside the GEMM launch (True, the default) or by a separate reduction launch (False; A/B):
    stc_set_splitk_inlaunch.  The workspace sizes and statistics chunk counts follow it, so the memoised queries
    are dropped.  Returns the previous setting."""
    old = bool(lib().stc_set_splitk_inlaunch(1 if on else 0))
    _MEMO.clear()
    return old


def plan_of(kind, B, gh, gw, cin, cout, dt):
    out = (ctypes.c_int32 * 4)()
    check(lib().stc_conv_fwd_plan(L.dtype_code(dt), kind, B, gh, gw, cin, cout, out), "stc_conv_fwd_plan")
    return tuple(out)


def conv(kind, B, xv, cin, w_packed, cout, yv, dt, pro=None, slope=None, bias=None, tanh=False, out_f32=False,
         force=None):
    """Implicit-GEMM conv family (stc_conv_fwd; force: a forced narrow-N tile through stc_conv_fwd_ex, tests)."""
    dev = w_packed.device
    if kind == L.CONVT_S2:
        gh, gw = xv.H, xv.W
    else:
        gh, gw = yv.H, yv.W
    l = lib()
    nbytes = _conv_ws_bytes(kind, B, gh, gw, cin, cout, dt)
    ws, nb = _ws(nbytes, dev)
    sc, sh = _pro(pro)
    timer = _timer
    if timer is not None:
        e0, e1 = _main_events()
    if force is not None:
        assert pro is None and slope is None
        rc = l.stc_conv_fwd_ex(L.dtype_code(dt), kind, B, xv, cin, ptr(w_packed), cout, yv, ptr(bias), int(tanh),
                               int(out_f32), None, 0, (ctypes.c_int32 * 2)(*force), ptr(ws), nb, stream())
    else:
        rc = l.stc_conv_fwd(L.dtype_code(dt), kind, B, xv, cin, sc, sh, 0 if slope is None else 1,
                            0.0 if slope is None else float(slope), ptr(w_packed), cout, yv, ptr(bias), int(tanh),
                            int(out_f32), ptr(ws), nb, stream())
    if timer is not None:
        _disarm()
    check(rc, "stc_conv_fwd")
    if timer is not None:
        _time_entry(timer, kind, B, gh, gw, cin, cout, dt, e0, e1)


def conv_query(kind, B, gh, gw, cin, cout, dt, out_f32=False, force=None):
    """(workspace bytes, stats chunks, plan (BM, BN, ksplit, narrow, cfg)) of stc_conv_fwd_ex."""
    key = ("cq", kind, B, gh, gw, cin, cout, dt, bool(out_f32), None if force is None else tuple(force))
    r = _MEMO.get(key)
    if r is not None:
        return r
    ws = ctypes.c_int64()
    nch = ctypes.c_int32()
    po = (ctypes.c_int32 * 5)()
    fp = (ctypes.c_int32 * 2)(*force) if force is not None else None
    check(lib().stc_conv_fwd_query(L.dtype_code(dt), kind, B, gh, gw, cin, cout, int(out_f32), fp, ctypes.byref(ws),
                                   ctypes.byref(nch), po), "stc_conv_fwd_query")
    r = _MEMO[key] = (ws.value, nch.value, tuple(po))
    return r


# Tuning hooks (scripts/train_steps.py --ab-plans): per-shape plan overrides of the forward convs with
# fused statistics, keyed (kind, B, gh, gw, cin, cout), and of the weight gradients, keyed
# (B, Hd, Wd, R, Cg); values {tile config, splits}.  Empty in production.
FORCE_CONV = {}
FORCE_WGRAD = {}


# conv + activation epilogue for the layers without BatchNorm (stc_conv_fwd_act); False (A/B scripts): conv +
# bn_apply
FUSE_ACT = True
# input-gradient conv + activation backward for the same layers (stc_conv_bwd_act); False (A/B, tests): conv +
# bn_backward(no table)
FUSE_ACT_BWD = True


def conv_act(kind, B, xv, cin, w_packed, cout, y1v, s1, dt, y2v=None, s2=0.0, bias=None):
    """Conv whose output goes straight through LeakyReLU/ReLU (no BatchNorm): y1 = act(out, s1) [and
    y2 = act(out, s2)] from the conv epilogue, bit-identical to conv + bn_apply(table None) without the raw
    tensor.  Returns False (nothing launched) when the shape has no such epilogue: the caller then runs the
    two-call form."""
    l = lib()
    y2 = y2v if y2v is not None else L.NULL_VIEW
    if not FUSE_ACT or dt != torch.bfloat16 or not l.stc_conv_fwd_act_ok(L.dtype_code(dt), kind, B, xv, cin, cout,
                                                                           y1v, y2):
        return False
    gh, gw = (xv.H, xv.W) if kind == L.CONVT_S2 else (y1v.H, y1v.W)
    dev = w_packed.device
    nbytes = _conv_ws_bytes(kind, B, gh, gw, cin, cout, dt)
    ws, nb = _ws(nbytes, dev)
    timer = _timer
    if timer is not None:
        e0, e1 = _main_events()
    rc = l.stc_conv_fwd_act(L.dtype_code(dt), kind, B, xv, cin, ptr(w_packed), cout, y1v, float(s1), y2, float(s2),
                            ptr(bias), ptr(ws), nb, stream())
    if timer is not None:
        _disarm()
    check(rc, "stc_conv_fwd_act")
    if timer is not None:
        # the 8-channel first layers run the streaming stem kernel (csrc/stem_bf16.hip, stem_eligible)
        stem = (kind == L.CONV_S2 and cin == 8 and cout == 64 and xv.W in (256, 512) and xv.co == 0 and xv.ps == 8
                and xv.H == 2 * gh and gh % 8 == 0)
        _time_entry(timer, kind, B, gh, gw, cin, cout, dt, e0, e1,
                    name=f"stem_conv_kernel<{xv.W}, {2 if y2v is not None else 1}>" if stem else None)
    return True


def conv_act_backward(kind, B, xv, cin, w_packed, cout, yv, dt, act_x, s_self, g_other=None, s_other=0.0):
    """Input-gradient conv (output yv) whose output reaches an activation with no BatchNorm: yv receives
    g_other*act'(x, s_other) + out*act'(x, s_self) (x = ``act_x``, the activation's input) from the conv epilogue,
    bit-identical to conv + bn_backward(no table) without the intermediate gradient tensor.  Returns False (nothing
    launched) when the layer has no such epilogue: the caller then runs the two-call form."""
    if not FUSE_ACT_BWD or dt != torch.bfloat16:
        return False
    l = lib()
    g2 = g_other if g_other is not None else L.NULL_VIEW
    key = ("actb", kind, B, cin, cout, L.layout_key(xv), L.layout_key(yv), L.layout_key(act_x),
           L.layout_key(g2) if g_other is not None else None)
    ok = _MEMO.get(key)
    if ok is None:
        ok = _MEMO[key] = bool(l.stc_conv_bwd_act_ok(L.dtype_code(dt), kind, B, xv, cin, cout, yv, act_x, g2))
    if not ok:
        return False
    timer = _timer
    if timer is not None:
        e0, e1 = _main_events()
    rc = l.stc_conv_bwd_act(L.dtype_code(dt), kind, B, xv, cin, ptr(w_packed), cout, yv, act_x, float(s_self), g2,
                            float(s_other), stream())
    if timer is not None:
        _disarm()
    check(rc, "stc_conv_bwd_act")
    if timer is not None:
        gh, gw = (xv.H, xv.W) if kind == L.CONVT_S2 else (yv.H, yv.W)
        _time_entry(timer, kind, B, gh, gw, cin, cout, dt, e0, e1, bnb=True)
    return True


def conv_stats(kind, B, xv, cin, w_packed, cout, yv, dt, bias=None, force=None):
    """Conv forward + fused BatchNorm partial statistics of its output (stc_conv_fwd_ex).
    Returns (part [chunks, cout, 4] fp32, chunks) for bn_finalize."""
    dev = w_packed.device
    gh, gw = (xv.H, xv.W) if kind == L.CONVT_S2 else (yv.H, yv.W)
    if force is None and FORCE_CONV:
        force = FORCE_CONV.get((kind, B, gh, gw, cin, cout))
    nbytes, nch, plan = conv_query(kind, B, gh, gw, cin, cout, dt, force=force)
    ws, nb = _ws(nbytes, dev)
    part = torch.empty((nch, cout, 4), dtype=torch.float32, device=dev)
    fp = (ctypes.c_int32 * 2)(*force) if force is not None else None
    timer = _timer
    if timer is not None:
        e0, e1 = _main_events()
    rc = lib().stc_conv_fwd_ex(L.dtype_code(dt), kind, B, xv, cin, ptr(w_packed), cout, yv, ptr(bias), 0, 0,
                               ptr(part), nch, fp, ptr(ws), nb, stream())
    if timer is not None:
        _disarm()
    check(rc, "stc_conv_fwd_ex")
    if timer is not None:
        _time_entry(timer, kind, B, gh, gw, cin, cout, dt, e0, e1)
    return part, nch


def conv_bn_act(kind, B, xv, cin, w_packed, cout, yv, dt, bn, apply_x, y1, s1, y2=None, s2=0.0, defer=None):
    """A BatchNorm layer's train-mode forward: conv into ``yv`` with the batch statistics, the BN finalize (running
    statistics updated) and the activation pass of ``apply_x`` into y1 [and y2] (y1 None: no pass) -- one library call
    (stc_conv_bn_fwd; the instrumented / forced-plan runs take the three separate calls).  Returns ((2, cout) scale /
    shift table, (mean, rstd)), views of one fp32 buffer.  defer (a list): the running statistics are left alone and
    (partials, chunks, cout, bn) is appended for bn_running_update."""
    dev = w_packed.device
    gh, gw = (xv.H, xv.W) if kind == L.CONVT_S2 else (yv.H, yv.W)
    upd = defer is None
    if _timer is not None or (FORCE_CONV and (kind, B, gh, gw, cin, cout) in FORCE_CONV):
        t = torch.empty((2, cout), dtype=torch.float32, device=dev)
        part, nch = conv_stats(kind, B, xv, cin, w_packed, cout, yv, dt)
        st = bn_finalize_part(part, nch, cout, bn, t[0], t[1], update_running=upd)
        if not upd:
            defer.append((part, nch, cout, bn))
        if y1 is not None:
            bn_apply(B, apply_x, cout, dt, (t[0], t[1]), y1, s1, y2, s2)
        return t, st
    nbytes, nch, _ = conv_query(kind, B, gh, gw, cin, cout, dt)
    ws, nb = _ws(nbytes, dev)
    P = nch * cout * 4
    fws = torch.empty(P + 4 * cout, dtype=torch.float32, device=dev)
    mom = bn.momentum if bn.momentum is not None else BN_MOMENTUM
    check(lib().stc_conv_bn_fwd(L.dtype_code(dt), kind, B, xv, cin, ptr(w_packed), cout, yv, ptr(fws), nch,
                                ptr(bn.weight), ptr(bn.bias), ptr(bn.running_mean) if upd else None,
                                ptr(bn.running_var) if upd else None, ptr(bn.num_batches_tracked) if upd else None,
                                float(mom), float(bn.eps),
                                apply_x if y1 is not None else L.NULL_VIEW, y1 if y1 is not None else L.NULL_VIEW,
                                float(s1), y2 if y2 is not None else L.NULL_VIEW, float(s2), ptr(ws), nb, stream()),
          "stc_conv_bn_fwd")
    if not upd:
        defer.append((fws, nch, cout, bn))
    tab = fws[P:]
    return tab[2 * cout:].view(2, cout), (tab[:cout], tab[cout:2 * cout])


def bn_running_update(part, nch, C, bn):
    """The running-statistics update a train-mode BatchNorm call left for later (conv_bn_act(defer=...)): the same
    finalize launch on the same partials (so the same mean / variance, bit for bit) with the running buffers this
    time, its table output discarded."""
    dev = part.device
    scratch = torch.empty(2 * C, dtype=torch.float32, device=dev)
    mom = bn.momentum if bn.momentum is not None else BN_MOMENTUM
    check(lib().stc_bn_finalize(ptr(part), nch, C, ptr(bn.weight), ptr(bn.bias), ptr(bn.running_mean),
                                ptr(bn.running_var), ptr(bn.num_batches_tracked), float(mom), float(bn.eps), None, None,
                                ptr(scratch), ptr(scratch[C:]), stream()), "stc_bn_finalize")


# bf16 LDS-DMA tile configurations (csrc/igemm_bf16.hip kTiles): cfg -> (BM, BN, WM, WN, stages, BK[, loader waves])
_BF16_TILES = [(128, 128, 2, 2, 2, 64), (256, 128, 2, 2, 2, 64), (128, 64, 2, 2, 2, 64), (256, 64, 4, 1, 2, 64),
               (64, 128, 1, 4, 2, 64), (64, 64, 2, 2, 2, 64), (256, 256, 2, 4, 2, 64), (128, 256, 2, 4, 2, 64),
               (128, 128, 2, 2, 3, 64), (128, 256, 2, 4, 3, 64), (64, 128, 1, 4, 3, 64), (128, 64, 2, 2, 3, 64),
               (64, 64, 2, 2, 3, 64), (256, 128, 4, 2, 3, 64), (256, 256, 2, 4, 4, 32), (256, 128, 4, 2, 4, 32),
               (128, 256, 2, 4, 4, 32), (128, 128, 2, 2, 4, 32), (128, 64, 2, 2, 4, 32), (64, 64, 2, 2, 4, 32),
               (128, 128, 2, 2, 3, 32), (128, 128, 2, 2, 2, 32), (256, 128, 4, 2, 3, 32), (128, 64, 2, 2, 3, 32),
               (128, 128, 2, 4, 2, 64), (128, 128, 4, 2, 2, 64), (128, 64, 4, 2, 2, 64), (256, 128, 4, 4, 2, 64),
               (128, 256, 4, 4, 2, 64), (128, 128, 2, 2, 4, 64, 4), (128, 128, 2, 2, 3, 64, 4),
               (256, 128, 4, 2, 3, 64, 4), (128, 64, 2, 2, 4, 64, 4), (128, 128, 2, 2, 2, 64, 2),
               (128, 64, 2, 2, 2, 64, 2), (128, 256, 2, 4, 2, 64, 2)]


# plan config of the conv-s2 halo kernel (stc_conv_fwd_query plan[4]; force_plan (HALO_CFG, 1) forces it)
HALO_CFG = 100


def kernel_name(kind, B, gh, gw, cin, cout, dt, bnb=False):
    """(kernel symbol as rocprof shows it, launches-a-single-kernel) of one conv call
    (bnb: the input-gradient form with the BatchNorm-backward reduction fused in)."""
    ws, _, plan = conv_query(kind, B, gh, gw, cin, cout, dt)
    bm, bn, ks, narrow, cfg = plan
    if narrow:
        if dt == torch.bfloat16 and cin % 64 == 0:
            geom = 0 if kind == L.CONVT_S2 else 1
            npc = 4 * cout if geom == 0 else cout
            nb = 2 if npc > 16 else 1
            # csrc/narrow_bf16.hip narrow_plan: the streaming ConvT kernel where it applies, else the 4x16 K-split tile
            if geom == 0 and gh % 16 == 0 and gw % 64 == 0 and ((cin == 128 and npc <= 16) or
                                                               (cin == 64 and 16 < npc <= 32)):
                return f"narrow_stream_kernel<{cin}, {nb}, {3 if cin == 128 else 4}>", True
            if geom == 1 and cout == 1 and cin in (256, 512):  # the two-pass logits form (taps GEMM + gather)
                return f"logits_taps_kernel<{cin}>", False
            return f"narrow_wk_kernel<{geom}, {nb}, 4, 1>", ws == 0
        return "narrow_tiled_kernel", True
    if cfg == HALO_CFG:  # the LDS-resident input halo kernels (csrc/halo_bf16.hip): template as rocprof names it
        convt = kind == L.CONVT_S2
        geom = {L.CONV_S2: 0, L.CONVT_S2: 1, L.CONV_S1: 2, L.CONV_S1_DGRAD: 3}[kind]
        vh, vw = (gh + 1, gw + 1) if kind == L.CONV_S1 else (gh, gw)  # (the s1 forward: its input grid)
        blocks = B * vh * vw // 256 * ((cout + bn - 1) // bn) * (4 if convt else 1)
        if bn == 64:  # (csrc/halo_bf16.hip halo_launch: conv-s2 grids <= 32 wide take the 8-wave 256 x 64 block)
            rb, wm, wn = (128, 8, 1) if (kind == L.CONV_S2 and vw <= 32) else (64, 4, 1)
            if convt and blocks // 2 >= 256:  # (the ConvT phase pair, GEOM 4: two phases per block)
                geom = 4
        else:
            rb, wm, wn = (64, 2, 2) if blocks >= 512 else (128, 4, 2)
        return (f"halo_conv_kernel<{geom}, {vw}, {bn}, {str(bnb).lower()}, {rb}, {wm}, {wn}>", True)
    if cfg >= 0:
        t = _BF16_TILES[cfg]
        if len(t) > 6:  # loader-wave blocks
            return (f"igemm_bf16_ld_kernel<{t[0]}, {t[1]}, {t[2]}, {t[3]}, {t[4]}, {t[5]}, {str(bnb).lower()}, {t[6]}>",
                    ks == 1)
        return f"igemm_bf16_kernel<{t[0]}, {t[1]}, {t[2]}, {t[3]}, {t[4]}, {t[5]}, {str(bnb).lower()}>", ks == 1
    tname = {torch.float32: "float", torch.bfloat16: "__hip_bfloat16"}[dt]
    return f"igemm_kernel<{tname}, {bm}, {bn}>", ks == 1


def _time_entry(timer, kind, B, gh, gw, cin, cout, dt, e0, e1, bnb=False, name=None):
    name, single = (name, True) if name else kernel_name(kind, B, gh, gw, cin, cout, dt, bnb)
    outs = B * gh * gw * (4 if kind == L.CONVT_S2 else 1)
    taps = 4 if kind == L.CONVT_S2 else 16
    timer.append((name, single, 2.0 * outs * cout * taps * cin, e0, e1,
                  f"{['conv_s2', 'conv_s1', 'convT', 's1_dgrad'][kind]} B{B} grid{gh}x{gw} cin{cin} cout{cout}"))


def conv_bn_backward(kind, B, xv, cin, w_packed, cout, yv, dt, bn_x, C, bn_state, gamma, s_self, ch_off=0,
                     g_other=None, s_other=0.0, dxv=None, dgamma=None, dbeta=None):
    """Input-gradient conv (output yv) whose output feeds a BatchNorm backward, with the BN
    reduction fused into the conv (stc_conv_bwd_bn), then the BN apply (stc_bn_bwd_apply):
    dx = BN-backward of dn = out*act'(n, s_self) [+ g_other*act'(n, s_other)].
    bn_state = (scale, shift, mean, rstd); returns (dgamma, dbeta) (written into ``dgamma``/``dbeta`` when given)."""
    dev = w_packed.device
    l = lib()
    gh, gw = (xv.H, xv.W) if kind == L.CONVT_S2 else (yv.H, yv.W)
    nbytes = _conv_ws_bytes(kind, B, gh, gw, cin, cout, dt)
    ws, nb = _ws(nbytes, dev)
    scale, shift, mean, rstd = bn_state
    fuse = L.BnbFuse(bn_x, g_other if g_other is not None else L.NULL_VIEW, scale.data_ptr(), shift.data_ptr(),
                     mean.data_ptr(), rstd.data_ptr(), float(s_self), float(s_other), C, ch_off)
    # the chunk count depends on which kernel takes the call, which depends on the views' layout (not only shapes)
    key = ("bnbch", kind, B, cin, cout, dt, L.layout_key(xv), L.layout_key(yv), bn_x.H, bn_x.W, g_other is None)
    nch = _MEMO.get(key)
    if nch is None:
        nch = _MEMO[key] = l.stc_conv_bwd_bn_chunks_ex(L.dtype_code(dt), kind, B, xv, cin, cout, yv,
                                                       ctypes.byref(fuse))
        check(0 if nch > 0 else -1, "stc_conv_bwd_bn_chunks_ex")
    part = torch.empty((nch, C, 2), dtype=torch.float32, device=dev)
    timer = _timer
    dgamma = _out1(dgamma, C, dev)
    dbeta = _out1(dbeta, C, dev)
    if timer is None:  # (both launches from one call)
        check(l.stc_conv_bwd_bn_apply(L.dtype_code(dt), kind, B, xv, cin, ptr(w_packed), cout, yv, ctypes.byref(fuse),
                                      ptr(part), nch, ptr(gamma), dxv, ptr(dgamma), ptr(dbeta), ptr(ws), nb, stream()),
              "stc_conv_bwd_bn_apply")
        return dgamma, dbeta
    e0, e1 = _main_events()
    rc = l.stc_conv_bwd_bn(L.dtype_code(dt), kind, B, xv, cin, ptr(w_packed), cout, yv, ctypes.byref(fuse),
                           ptr(part), nch, ptr(ws), nb, stream())
    _disarm()
    check(rc, "stc_conv_bwd_bn")
    _time_entry(timer, kind, B, gh, gw, cin, cout, dt, e0, e1, bnb=yv.cs == 1)
    # apply: g1 = the conv output at the BN channels over the BN extent
    g1 = L.View(yv.p, bn_x.H, bn_x.W, yv.bs, yv.rs, yv.ps, yv.co + ch_off, yv.cs, 0)
    g1._keep = yv
    check(l.stc_bn_bwd_apply(L.dtype_code(dt), B, bn_x, C, ptr(scale), ptr(shift), ptr(mean), ptr(rstd), ptr(gamma),
                             g1, float(s_self), g_other if g_other is not None else L.NULL_VIEW, float(s_other),
                             ptr(part), nch, dxv, ptr(dgamma),
                             ptr(dbeta), stream()), "stc_bn_bwd_apply")
    return dgamma, dbeta


def bn_finalize_part(part, nch, C, bn, scale_out, shift_out, update_running=True):
    """mean/rstd + (scale, shift) table from conv_stats partials; updates running stats."""
    dev = scale_out.device
    mean = torch.empty(C, dtype=torch.float32, device=dev)
    rstd = torch.empty(C, dtype=torch.float32, device=dev)
    rm = bn.running_mean if update_running else None
    rv = bn.running_var if update_running else None
    nbt = bn.num_batches_tracked if update_running else None
    mom = bn.momentum if bn.momentum is not None else BN_MOMENTUM
    check(lib().stc_bn_finalize(ptr(part), nch, C, ptr(bn.weight), ptr(bn.bias), ptr(rm), ptr(rv), ptr(nbt),
                                float(mom), float(bn.eps), ptr(mean), ptr(rstd), ptr(scale_out), ptr(shift_out),
                                stream()), "stc_bn_finalize")
    return mean, rstd


# bf16 weight-gradient tile configurations (csrc/wgrad_bf16.hip kWbCfg): cfg -> (BM, BN, WM, WN, swapped)
_WB_TILES = [(128, 128, 2, 2, "false"), (64, 128, 1, 4, "false"), (128, 16, 4, 1, "true"), (256, 256, 2, 4, "false"),
             (256, 128, 4, 2, "false"), (128, 256, 2, 4, "false"), (128, 128, 2, 2, "false", 4, 4),
             (128, 128, 2, 2, "false", 4, 3),
             (128, 256, 2, 2, "false", -2, 4)]  # (BM, BN, WM, WN, swapped[, loader waves (-2: halo), stages])


def wgrad_query(B, Hd, Wd, R, Cg, dt, force=None):
    """(workspace bytes, plan (cfg, BM, BN, splits, slab)) of stc_conv_wgrad_ex for these arguments."""
    key = ("wq", B, Hd, Wd, R, Cg, dt, None if force is None else tuple(force))
    r = _MEMO.get(key)
    if r is not None:
        return r
    ws = ctypes.c_int64()
    po = (ctypes.c_int32 * 5)()
    fp = (ctypes.c_int32 * 2)(*force) if force is not None else None
    check(lib().stc_conv_wgrad_query(L.dtype_code(dt), B, Hd, Wd, R, Cg, fp, ctypes.byref(ws), po),
          "stc_conv_wgrad_query")
    r = _MEMO[key] = (ws.value, tuple(po))
    return r


def _wgrad_kernel_name(plan, Hd, Wd):
    cfg = plan[0]
    if cfg < 0:
        return "wgrad_kernel"
    bm, bn, wm, wn, sw = _WB_TILES[cfg][:5]
    ld, nst = _WB_TILES[cfg][5:] if len(_WB_TILES[cfg]) > 5 else (0, 2)
    ghw = Hd * Wd
    pow2 = lambda v: v > 0 and (v & (v - 1)) == 0  # noqa: E731
    fast = Wd % 64 == 0 or (pow2(Wd) and ghw % 64 == 0) or (pow2(ghw) and pow2(Wd) and 64 % ghw == 0)
    fast = fast and cfg != 3  # the 256x256 tile keeps the general addressing (register budget)
    if ld == -2:  # (the stride-1 halo tile: a 31-wide grid run as 32 x 32)
        return "wgrad_halo_kernel<32, true>" if Wd == 31 else f"wgrad_halo_kernel<{min(Wd, 64)}, false>"
    if ld:
        return f"wgrad_bf16_ld_kernel<{bm}, {bn}, {wm}, {wn}, {sw}, {str(fast).lower()}, {ld}, {nst}>"
    return f"wgrad_bf16_kernel<{bm}, {bn}, {wm}, {wn}, {sw}, {str(fast).lower()}>"


# The narrow-R weight gradient (stc_conv_wgrad_rows) for the PatchGAN logits layer: bf16 on the MFMA rows kernel
# (11 + 5 us with its ordered reduce, bs=32), fp32 on the VALU rows kernel (non-packed v_fma_f32: compiled to
# v_pk_fma_f32 with op_sel it returned sporadically different low-half sums with two processes on one GPU,
# tests/test_gpu_dist.py); ~75 us for the padded GEMM.  rows_kernel=False per call takes the GEMM path.
_ROWS_DEFAULT = True


def _out1(t, n, device):
    """A caller-provided fp32 output of n elements (e.g. a view of a flat gradient buffer), or a new one."""
    if t is None:
        return torch.empty(n, dtype=torch.float32, device=device)
    assert t.dtype == torch.float32 and t.is_contiguous() and t.numel() == n, "output: fp32, contiguous, n elements"
    return t


def _out_w(t, R, Cg_out, device):
    if t is None:
        return torch.empty((R, Cg_out, 4, 4), dtype=torch.float32, device=device)
    assert t.dtype == torch.float32 and t.is_contiguous() and tuple(t.shape) == (R, Cg_out, 4, 4), \
        f"wgrad output: fp32 contiguous [{R}, {Cg_out}, 4, 4], got {tuple(t.shape)}"
    return t


def wgrad(B, stride, Dv, R, Gv, Cg, Cg_out, dt, dpro=None, dslope=None, gpro=None, gslope=None, device=None,
          force=None, rows=None, rows_kernel=None, out=None):
    """Weight gradient [R][Cg_out][4][4] fp32 (stc_conv_wgrad_ex; force = optional {tile config, splits}),
    written into ``out`` when given (e.g. a view of a flat gradient buffer).
    rows: the number of nonzero (real) channels of D when the rest is padding -- a stride-1 layer with
    1-2 of them goes to stc_conv_wgrad_rows (which then writes only R = ``rows`` rows when R == rows)."""
    l = lib()
    if (rows is not None and rows <= 2 and stride == 1 and (_ROWS_DEFAULT if rows_kernel is None else rows_kernel) and dpro is None and gpro is None and dslope is None
            and gslope is None and force is None and Cg % 64 == 0 and ((Dv.H + 4) * (Dv.W + 4) + 16384) * rows <= 40000):
        nbytes = l.stc_conv_wgrad_rows_workspace(B, Gv.H, rows, Cg)
        ws, nb = _ws(nbytes, device)
        if out is not None and out.shape[0] == rows:  # only the real rows (e.g. straight into a gradient view)
            R = rows
        dW = _out_w(out, R, Cg_out, device)
        timer = _timer
        if timer is not None:
            e0, e1 = _main_events()
        rc = l.stc_conv_wgrad_rows(L.dtype_code(dt), B, Dv, R, rows, Gv, Cg, Cg_out, ptr(dW), ptr(ws), nb, stream())
        if timer is not None:
            _disarm()
        check(rc, "stc_conv_wgrad_rows")
        if timer is not None:
            timer.append(("wgrad_rows_kernel", True, 2.0 * B * Dv.H * Dv.W * R * 16 * Cg, e0, e1,
                          f"wgrad s1 P={B * Dv.H * Dv.W} R{R} (real {rows}) Cg{Cg}"))
        return dW
    if out is not None and out.shape[0] != R:  # real rows of a padded R: through a scratch
        full = wgrad(B, stride, Dv, R, Gv, Cg, Cg_out, dt, dpro, dslope, gpro, gslope, device, force)
        out.copy_(full[:out.shape[0]])
        return out
    if force is None and FORCE_WGRAD:
        force = FORCE_WGRAD.get((B, Dv.H, Dv.W, R, Cg))
    nbytes, plan = wgrad_query(B, Dv.H, Dv.W, R, Cg, dt, force)
    ws, nb = _ws(nbytes, device)
    dW = _out_w(out, R, Cg_out, device)
    dsc, dsh = _pro(dpro)
    gsc, gsh = _pro(gpro)
    fp = (ctypes.c_int32 * 2)(*force) if force is not None else None
    timer, ctimer = _timer, _call_timer
    if timer is not None:
        e0, e1 = _main_events()
    if ctimer is not None:
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record()
    rc = l.stc_conv_wgrad_ex(L.dtype_code(dt), B, stride, Dv, R, dsc, dsh, 0 if dslope is None else 1,
                             0.0 if dslope is None else float(dslope), Gv, Cg, Cg_out, gsc, gsh,
                             0 if gslope is None else 1, 0.0 if gslope is None else float(gslope), ptr(dW), fp,
                             ptr(ws), nb, stream())
    if ctimer is not None:
        c1.record()
    if timer is not None:
        _disarm()
    check(rc, "stc_conv_wgrad_ex")
    if timer is not None or ctimer is not None:
        dma = dt == torch.bfloat16 and dpro is None and gpro is None and dslope is None and gslope is None
        name = _wgrad_kernel_name(plan, Dv.H, Dv.W) if dma else "wgrad_kernel"
    if ctimer is not None:
        ctimer.append((name, c0, c1))
    if timer is not None:
        timer.append((name, not plan[4], 2.0 * B * Dv.H * Dv.W * R * 16 * Cg, e0, e1,
                      f"wgrad s{stride} P={B * Dv.H * Dv.W} R{R} Cg{Cg}"))
    return dW


_PHASED = {L.PACK_CONV_DGRAD, L.PACK_CONVT_FWD}


# bumped whenever a packed-operand buffer is created or dropped: the optimiser's cached pointer tables
# (optim.Adam._fast_step) hold the addresses of these buffers
PACK_EPOCH = 0


def invalidate_packs():
    global PACK_EPOCH
    PACK_EPOCH += 1


def pack(mode, W, n_pad, c_pad, dt):
    """Pack a torch weight [P][Q][4][4] into the GEMM operand layout [phases][n_pad][taps][c_pad]."""
    invalidate_packs()
    P, Q = W.shape[0], W.shape[1]
    nph, taps = (4, 4) if mode in _PHASED else (1, 16)
    out = torch.empty((nph, n_pad, taps, c_pad), dtype=dt, device=W.device)
    Wc = W.detach()
    if not Wc.is_contiguous():
        Wc = Wc.contiguous()
    check(lib().stc_pack_weight(L.dtype_code(dt), mode, ptr(Wc), P, Q, ptr(out), n_pad, c_pad, stream()),
          "stc_pack_weight")
    return out


# generation counter bumped by our optimizer (it updates parameters in place behind autograd's back)
_GEN = {}
# id(weight) -> {cache key: cache} of every packed operand made from it (the optimizer rewrites
# them in the same pass as the update: stc_adam_pack_step)
_PACK_OWNERS = {}


def pack_version(W):
    return (W._version, _GEN.get(id(W), 0), W.data_ptr())


def pack_targets(W):
    """[(key, cache, mode, out, n_pad, c_pad, dtype)] of the packed operands of weight W."""
    out = []
    for key, cache in _PACK_OWNERS.get(id(W), {}).items():
        hit = cache.get(key)
        if hit is None:
            continue
        _, mode, n_pad, c_pad, dt = cache["__keys__"][key]
        out.append((key, cache, mode, hit[1], n_pad, c_pad, dt))
    return out


def bump(params):
    for p in params:
        _GEN[id(p)] = _GEN.get(id(p), 0) + 1


def packed(cache, W, mode, n_pad, c_pad, dt):
    """Cached packed weight; repacked when the parameter changed (version or optimizer step).
    Every key is remembered so that refresh_packs() can repack all stale ones in one launch."""
    key = (id(W), mode, n_pad, c_pad, dt)
    ver = (W._version, _GEN.get(id(W), 0), W.data_ptr())
    hit = cache.get(key)
    if hit is not None and hit[0] == ver:
        return hit[1]
    cache.setdefault("__keys__", {})[key] = (W, mode, n_pad, c_pad, dt)
    _PACK_OWNERS.setdefault(id(W), {})[key] = cache
    t = pack(mode, W, n_pad, c_pad, dt)
    cache[key] = (ver, t)
    return t


def refresh_packs(cache):
    """Repack every stale cached operand of a network (after an optimiser step) with one
    multi-tensor launch per dtype (stc_pack_weights), reusing the packed buffers in place."""
    keys = cache.get("__keys__")
    if not keys:
        return
    jobs = {}
    for key, (W, mode, n_pad, c_pad, dt) in keys.items():
        ver = (W._version, _GEN.get(id(W), 0), W.data_ptr())
        hit = cache.get(key)
        if hit is not None and hit[0] == ver:
            continue
        if hit is None:
            nph, taps = (4, 4) if mode in _PHASED else (1, 16)
            out = torch.empty((nph, n_pad, taps, c_pad), dtype=dt, device=W.device)
            invalidate_packs()
        else:
            out = hit[1]
        Wc = W.detach()
        assert Wc.is_contiguous()
        jobs.setdefault(dt, []).append((L.PackDesc(mode, W.shape[0], W.shape[1], n_pad, c_pad, 0, Wc.data_ptr(),
                                                   out.data_ptr()), key, ver, out))
    for dt, lst in jobs.items():
        for i in range(0, len(lst), L.PACK_MAX):
            chunk = lst[i:i + L.PACK_MAX]
            arr = (L.PackDesc * len(chunk))(*[c[0] for c in chunk])
            check(lib().stc_pack_weights(L.dtype_code(dt), len(chunk), arr, stream()), "stc_pack_weights")
            for _, key, ver, out in chunk:
                cache[key] = (ver, out)


def stats_chunks(B, H, W):
    return lib().stc_chan_stats_chunks(B, H, W)


def bn_train_table(B, xv, C, dt, bn, scale_out, shift_out, update_running=True):
    """Batch statistics of x (view, C channels) -> (mean, rstd); writes the prologue table
    scale_out/shift_out (views of C floats) and updates bn's running statistics."""
    dev = scale_out.device
    nch = stats_chunks(B, xv.H, xv.W)
    part = torch.empty((nch, C, 4), dtype=torch.float32, device=dev)
    check(lib().stc_chan_stats(L.dtype_code(dt), B, xv, C, ptr(part), nch, stream()), "stc_chan_stats")
    mean = torch.empty(C, dtype=torch.float32, device=dev)
    rstd = torch.empty(C, dtype=torch.float32, device=dev)
    rm = bn.running_mean if update_running else None
    rv = bn.running_var if update_running else None
    nbt = bn.num_batches_tracked if update_running else None
    mom = bn.momentum if bn.momentum is not None else BN_MOMENTUM
    check(lib().stc_bn_finalize(ptr(part), nch, C, ptr(bn.weight), ptr(bn.bias), ptr(rm), ptr(rv), ptr(nbt),
                                float(mom), float(bn.eps), ptr(mean), ptr(rstd), ptr(scale_out), ptr(shift_out),
                                stream()), "stc_bn_finalize")
    return mean, rstd


def bn_eval_table(C, bn, scale_out, shift_out):
    check(lib().stc_bn_finalize(None, 0, C, ptr(bn.weight), ptr(bn.bias), ptr(bn.running_mean),
                                ptr(bn.running_var), None, 0.0, float(bn.eps), None, None, ptr(scale_out),
                                ptr(shift_out), stream()), "stc_bn_finalize(eval)")


def bn_apply(B, xv, C, dt, table, y1, s1, y2=None, s2=1.0):
    """y1 = act(x*scale+shift, s1) [, y2 = act(.., s2)]; table = (scale, shift) or None (identity)."""
    sc, sh = _pro(table)
    check(lib().stc_bn_apply(L.dtype_code(dt), B, xv, C, sc, sh, y1, float(s1),
                             y2 if y2 is not None else L.NULL_VIEW, float(s2), stream()), "stc_bn_apply")


def bn_backward(B, xv, C, dt, dxv, g1=None, s1=0.0, g2=None, s2=0.0, bn_state=None, dgamma=None, dbeta=None):
    """Fused activation + BatchNorm backward.  bn_state = (scale, shift, mean, rstd, gamma) or None
    (no BN: dx = g1*act1'(x) + g2*act2'(x)).  Returns (dgamma, dbeta) or (None, None)."""
    l = lib()
    g1v = g1 if g1 is not None else L.NULL_VIEW
    g2v = g2 if g2 is not None else L.NULL_VIEW
    dev_t = None
    if bn_state is None:
        check(l.stc_bn_bwd_apply(L.dtype_code(dt), B, xv, C, None, None, None, None, None, g1v, float(s1), g2v,
                                 float(s2), None, 0, dxv, None, None, stream()), "stc_bn_bwd_apply")
        return None, None
    scale, shift, mean, rstd, gamma = bn_state
    dev_t = scale.device
    nch = stats_chunks(B, xv.H, xv.W)
    part = torch.empty((nch, C, 2), dtype=torch.float32, device=dev_t)
    check(l.stc_bn_bwd_reduce(L.dtype_code(dt), B, xv, C, ptr(scale), ptr(shift), ptr(mean), ptr(rstd), g1v,
                              float(s1), g2v, float(s2), ptr(part), nch, stream()), "stc_bn_bwd_reduce")
    dgamma = _out1(dgamma, C, dev_t)
    dbeta = _out1(dbeta, C, dev_t)
    check(l.stc_bn_bwd_apply(L.dtype_code(dt), B, xv, C, ptr(scale), ptr(shift), ptr(mean), ptr(rstd), ptr(gamma),
                             g1v, float(s1), g2v, float(s2), ptr(part), nch, dxv, ptr(dgamma), ptr(dbeta), stream()),
          "stc_bn_bwd_apply")
    return dgamma, dbeta


def chan_sum(B, xv, C, Cout, dt, device, out=None):
    nch = stats_chunks(B, xv.H, xv.W)
    part = torch.empty((nch, C), dtype=torch.float32, device=device)
    out = _out1(out, Cout, device)
    check(lib().stc_chan_sum(L.dtype_code(dt), B, xv, C, Cout, ptr(part), nch, ptr(out), stream()), "stc_chan_sum")
    return out


def tanh_bias_bwd(y, gy, dqv, dt, dbias=None):
    """dq = gy*(1-y^2) into the NHWC view dqv (padded channels zero); returns dbias [C] (into ``dbias``
    when given)."""
    B, C, H, W = y.shape
    nch = stats_chunks(B, H, W)
    part = torch.empty((nch, C), dtype=torch.float32, device=y.device)
    dbias = _out1(dbias, C, y.device)
    check(lib().stc_tanh_bias_bwd(L.dtype_code(dt), B, C, H, W, ptr(y), ptr(gy), dqv, ptr(dbias), ptr(part), nch,
                                  stream()), "stc_tanh_bias_bwd")
    return dbias


def gather(sources, dst, dt):
    """NCHW fp32 sources (channel concat) -> NHWC dst [B, H, W, Cpad] (extra channels zero)."""
    B, H, W, cpad = dst.shape
    n = len(sources)
    arr = (ctypes.c_void_p * n)(*[s.data_ptr() for s in sources])
    cs = (ctypes.c_int * n)(*[s.shape[1] for s in sources])
    check(lib().stc_gather_nchw(L.dtype_code(dt), B, H, W, n, arr, cs, L.nhwc_view(dst), cpad, stream()),
          "stc_gather_nchw")


def scatter(src_nhwc, dsts, chans, dt, H=None, W=None):
    """NHWC -> NCHW fp32 per channel range; dsts entries may be None (skipped)."""
    B, Ha, Wa, _ = src_nhwc.shape
    H = Ha if H is None else H
    W = Wa if W is None else W
    n = len(dsts)
    arr = (ctypes.c_void_p * n)(*[None if d is None else d.data_ptr() for d in dsts])
    cs = (ctypes.c_int * n)(*chans)
    check(lib().stc_scatter_nchw(L.dtype_code(dt), B, H, W, L.nhwc_view(src_nhwc, 0, H, W), n, arr, cs, stream()),
          "stc_scatter_nchw")


def infer_output(net_out, oh=192, ow=256):
    """STCGAN.infer output stage on the GPU (stc_infer_output): generator output [B, C, H, W] fp32
    (tanh range) -> uint8 [B, oh, ow, C] = float2uint(cv.resize(x*0.5+0.5, (ow, oh), INTER_LINEAR)),
    the arrays the reference hands to cv.imwrite (STCGAN/stcgan.py:355-377, utils.py:63-65)."""
    if not net_out.is_cuda:
        raise RuntimeError("stcgan_amd.infer_output: CUDA (HIP) tensors only")
    x = net_out.detach().float().contiguous()
    B, C, H, W = x.shape
    out = torch.empty((B, oh, ow, C), dtype=torch.uint8, device=x.device)
    check(lib().stc_infer_output(ptr(x), B, C, H, W, oh, ow, ptr(out), stream()), "stc_infer_output")
    return out


def grad_accumulate(pairs):
    """dst += src (fp32, contiguous, same numel) for every (dst, src) in pairs: one launch per 16."""
    for k in range(0, len(pairs), 16):
        chunk = pairs[k:k + 16]
        for d, s in chunk:
            assert d.dtype == torch.float32 and s.dtype == torch.float32 and d.is_contiguous() \
                and s.is_contiguous() and d.numel() == s.numel(), "grad_accumulate: fp32 contiguous pairs"
        n = len(chunk)
        dst = (ctypes.c_void_p * n)(*[d.data_ptr() for d, _ in chunk])
        src = (ctypes.c_void_p * n)(*[s.data_ptr() for _, s in chunk])
        num = (ctypes.c_int64 * n)(*[d.numel() for d, _ in chunk])
        check(lib().stc_grad_accumulate(n, dst, src, num, stream()), "stc_grad_accumulate")
