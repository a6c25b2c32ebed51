#!/usr/bin/env python
"""ST-CGAN train-step benchmark on MI355X (BASELINE.json metric).

A "step" is one full ST-CGAN training iteration (STCGAN.run_epoch body,
STCGAN/stcgan.py:208-312): 6 network forwards + D backward + Adam(D), then 4
discriminator forwards + G backward + Adam(G), on a resident synthetic batch of
256x256 triplets (x, y ~ U(-1,1), m = +-1), batch 32 per GPU (BASELINE config 3/4).
Multi-GPU: one process per GPU, batch sharded (32 per rank, weak scaling), RCCL
all-reduce of the G/D gradients.  ``--gpus N`` with N > 1 and no torchrun environment
starts the N rank processes itself (a child ``torch.distributed.run``, launched before
this process touches the GPU) and relays rank 0's line.

Prints ONE JSON line on rank 0 (the driver contract), with:
  roofline      the dominant kernel by summed device time over every conv-family launch of
                one train step (HIP events bracketing each MAIN kernel, not the reductions
                enqueued after it), its algorithmic TFLOP/s vs the bf16/fp32 MFMA peak, its HBM
                bytes per launch from the committed rocprofv3 PMC passes; the whole step's and
                the north-star G1+G2 forward's MFMA fractions;
  parity        the metric's "G2 max-abs vs CPU": G1 -> G2 at ngf=64 (256x256) on this GPU vs the
                CPU oracle, fp32 (BASELINE target 1e-4) and bf16;
  configs       the other BASELINE configs' throughput (C2 fp32 G1+G2 fwd+bwd bs=16, C5 480x640
                inference bs=8);
  cpu_baseline  the oracle (a torch-CPU restatement of the reference, pinned by the reference's
                goldens) on this host's cores at BASELINE's units (C3 bs=32 step; C1, C2, C5).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
sys.path.insert(0, ROOT)

METRIC = "ST-CGAN train images/s at 256×256 bs=32, 1/2/4/8 MI355X; G2 max-abs vs CPU"
PEAK_TFLOPS = {"fp32": 157.3, "bf16": 2516.0}  # MI355X dense MFMA (MI355X_MICROARCH.md)
STEP_GFLOP_PER_IMG = 186.23  # conv + convT fwd/bwd FLOPs of one train step
# the PatchGAN logits conv (512 -> 1, k4 s1, 30 x 30 outputs) of the G step's two real-input discriminator calls,
# which loss type "normal" skips (engine stats_only): 2 x 2 x 900 x 16 x 512 FLOP per image
SKIPPED_LOGITS_GFLOP_PER_IMG = 2 * 2 * 900 * 16 * 512 / 1e9


def gen_fwd_flops(in_c, out_c, ngf, B, H, W, num_downs=8):
    """Algorithmic FLOPs (2*MAC) of one U-Net generator forward (real channels, no padding)."""
    co = [ngf * min(2 ** k, 8) for k in range(num_downs)]
    S = [(H, W), (H // 2, W // 2)]
    for _ in range(2, num_downs + 1):
        S.append(((S[-1][0] + 1) // 2, (S[-1][1] + 1) // 2))
    f = 0
    for k in range(num_downs):
        cin = in_c if k == 0 else co[k - 1]
        f += 2 * B * S[k + 1][0] * S[k + 1][1] * co[k] * 16 * cin
    for k in range(num_downs):
        cin = co[k] if k == num_downs - 1 else 2 * co[k]
        cout = out_c if k == 0 else co[k - 1]
        f += 2 * B * (2 * S[k + 1][0]) * (2 * S[k + 1][1]) * cout * 4 * cin
    return f


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="per-GPU batch")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--ngf", type=int, default=64)
    ap.add_argument("--dtype", default=os.environ.get("STC_BENCH_DTYPE", "bf16"), choices=["fp32", "bf16"])
    ap.add_argument("--graph", action="store_true", help="replay the step captured as one HIP graph "
                    "(STCGAN.capture; the same kernels, bit-identical results) instead of eager steps")
    ap.add_argument("--no-lanes", action="store_true", help="discriminators on the main stream (no side lanes; A/B)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the parity / other-config measurements")
    ap.add_argument("--cpu-batch", type=int, default=32, help="batch of the timed CPU train step (C3: 32)")
    return ap.parse_args()


def spawn_ranks(n):
    """--gpus N > 1 without a torchrun environment: run N rank processes (one per GPU) under
    torch.distributed.run as a CHILD process -- started before this process touches the GPU, so
    nothing is exec'd from an initialised process -- and relay its output and exit code."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def host_cores():
    """Cores this process may use: the affinity set, capped by a cgroup CPU quota if one is set."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = max(1, min(n, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(args):
    """The CPU oracle (oracle/stcgan_ref.py, a torch-CPU restatement of the reference run_epoch,
    parity-pinned by tests/golden) on this host's cores, at BASELINE's units: C3 = one full train
    step at batch 32, two timed iterations after one warm-up step at batch 4, plus C1 (G1 forward bs=4,
    under torch.no_grad), C2 (G1+G2 forward+backward bs=16) and C5 (480x640 G1->G2 inference bs=8)."""
    import torch
    from oracle import stcgan_ref as ref
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from fixture_init import fixture_state, pm_one, uniform
    threads = host_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    ngf, s = args.ngf, args.size
    states = {
        "G1": fixture_state(ref.generator_state_template(3, 1, ngf), 11, "ref"),
        "G2": fixture_state(ref.generator_state_template(4, 3, ngf), 12, "ref"),
        "D1": fixture_state(ref.discriminator_state_template(4, ngf), 13, "ref"),
        "D2": fixture_state(ref.discriminator_state_template(7, ngf), 14, "ref"),
    }
    tr = ref.OracleSTCGAN(states)

    def batch(bs):
        return [([], uniform((bs, 3, s, s), 1), pm_one((bs, 1, s, s), 2), uniform((bs, 3, s, s), 3))]

    t_all = time.perf_counter()
    tr.run_epoch(batch(4))  # warm-up (allocator, kernels)
    bs = args.cpu_batch
    b = batch(bs)
    t0 = time.perf_counter()
    for _ in range(2):
        tr.run_epoch(b)
    c3 = 2 * bs / (time.perf_counter() - t0)
    # C1: G1 forward bs=4 (train-mode BN), 2 timed iterations
    x4 = uniform((4, 3, s, s), 4)
    with torch.no_grad():
        t0 = time.perf_counter()
        for _ in range(2):
            ref.generator_forward(states["G1"], x4, True)
        c1 = 8 / (time.perf_counter() - t0)
    # C2: G1 + G2 forward + backward (L1 data losses) bs=16, 1 timed iteration
    x16, m16, y16 = uniform((16, 3, s, s), 5), pm_one((16, 1, s, s), 6), uniform((16, 3, s, s), 7)
    t0 = time.perf_counter()
    mp = ref.generator_forward(states["G1"], x16, True)
    yp = ref.generator_forward(states["G2"], torch.cat((x16, mp), 1), True)
    (ref.data_loss(mp, m16) + 5 * ref.data_loss(yp, y16)).backward()
    c2 = 16 / (time.perf_counter() - t0)
    # C5: 480x640 eval-mode inference bs=8
    x8 = uniform((8, 3, 480, 640), 8)
    with torch.no_grad():
        t0 = time.perf_counter()
        mp = ref.generator_forward(states["G1"], x8, False)
        ref.generator_forward(states["G2"], torch.cat((x8, mp), 1), False)
        c5 = 8 / (time.perf_counter() - t0)
    total = time.perf_counter() - t_all
    torch.set_num_threads(prev)
    return {"value": round(c3, 4), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"oracle run_epoch (full D+G train step, fp32, ngf={ngf}) at batch {bs} {s}x{s}: two "
                      f"timed iterations after a batch-4 warm-up; C1 is the G1 forward under torch.no_grad "
                      f"(train-mode BatchNorm, 2 iterations); whole CPU leg {total:.1f} s",
            "configs": {"C1_g1_fwd_bs4_img_s": round(c1, 3), "C2_g1g2_fwd_bwd_bs16_img_s": round(c2, 3),
                        "C3_train_step_bs32_img_s": round(c3, 4), "C5_infer_480x640_bs8_img_s": round(c5, 3)}}


def make_trainer(ngf, dtype, local):
    import types
    from stcgan_amd.stcgan import STCGAN
    a = types.SimpleNamespace(devices=[f"cuda:{local}"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5,
                              beta2=0.999, D_loss_fn="standard", D_loss_type="normal", ngf=ngf,
                              dtype=dtype, load_weights_g1=None, load_weights_g2=None,
                              load_weights_d1=None, load_weights_d2=None)
    return STCGAN(a)


def alg_bytes(name, desc):
    """Algorithmic HBM bytes of one GEMM-family launch (bf16 operands): the input, the output and the weights once
    (weight gradients: both operands once + the fp32 gradient; the fused BatchNorm-backward epilogue also reads
    the BN input and the second gradient, output-sized), from the timer's description (ops._time_entry)."""
    import re
    g = {k: int(v) for k, v in re.findall(r"(B|grid|cin|cout|P=|R|Cg)(\d+)", desc.replace("x", " x"))}
    if desc.startswith("wgrad"):
        P, R, C = g["P="], g["R"], g["Cg"]
        return 2 * P * R + 2 * (4 if " s2 " in desc else 1) * P * C + 4 * 16 * R * C
    gh, gw = (int(v) for v in re.search(r"grid(\d+)x(\d+)", desc).groups())
    B, cin, cout = g["B"], g["cin"], g["cout"]
    kind = desc.split()[0]
    outs = {"conv_s2": (B * 4 * gh * gw, B * gh * gw), "conv_s1": (B * (gh + 1) * (gw + 1), B * gh * gw),
            "s1_dgrad": (B * (gh - 1) * (gw - 1), B * gh * gw), "convT": (B * gh * gw, B * 4 * gh * gw)}[kind]
    byt = 2 * outs[0] * cin + 2 * outs[1] * cout + 2 * 16 * cin * cout
    if "true" in name.split("<", 1)[-1]:  # (BNB: the BN input and the other gradient)
        byt += 2 * 2 * outs[1] * cout
    return byt


def roofline_of_step(tr, x, m, y, args, B, s):
    """Dominant kernel of one (untimed) train step by summed device time, and the north-star set."""
    import torch
    from stcgan_amd import engine, ops
    def timed_step(single):
        # single: one stream (no side-stream networks or weight gradients), so each launch's events bracket
        # it alone; else the bench's own overlapped step (in situ: kernels share the GPU with the lanes')
        ops._timer, ops._call_timer = [], []
        lanes, overlap = tr.streams, engine.WGRAD_OVERLAP
        if single:
            tr.streams, engine.WGRAD_OVERLAP = False, False
        tr.train_step(x, m, y)
        torch.cuda.synchronize()
        launches, ops._timer = ops._timer, None
        calls, ops._call_timer = ops._call_timer, None
        tr.streams, engine.WGRAD_OVERLAP = lanes, overlap
        per, shapes = {}, {}
        for name, _single, fl, e0, e1, desc in launches:
            ms = e0.elapsed_time(e1)
            a = per.setdefault(name, [0, 0.0, 0.0, 0.0])
            a[0] += 1
            a[1] += fl
            a[2] += ms
            a[3] += alg_bytes(name, desc)
            shapes.setdefault(name, []).append((round(ms * 1e3, 1), desc))
        whole = {}  # weight-gradient calls: main kernel + split-pixel reduction
        for name, c0, c1 in calls:
            whole[name] = whole.get(name, 0.0) + c0.elapsed_time(c1)
        timed_step.whole = whole
        return launches, per, shapes

    launches, per, shapes = timed_step(True)
    whole_single = dict(timed_step.whole)
    dom = max(per, key=lambda k: per[k][2])
    n_dom, fl_dom, ms_dom, by_dom = per[dom]
    peak = PEAK_TFLOPS[args.dtype]
    achieved = fl_dom / (ms_dom * 1e-3) / 1e12
    _, per_situ, _ = timed_step(False)
    n_s, fl_s, ms_s, _ = per_situ.get(dom, (n_dom, fl_dom, float("nan"), 0.0))
    achieved_situ = fl_s / (ms_s * 1e-3) / 1e12
    # the largest consumer of the bench's own overlapped step (in situ, side streams on) may be another kernel
    dom_situ = max(per_situ, key=lambda k: per_situ[k][2])
    nd, fld, msd, _ = per_situ[dom_situ]
    situ_dominant = {"kernel": dom_situ, "launches": nd, "gflop": round(fld / 1e9, 2), "ms": round(msd, 3),
                     "avg_us": round(msd / nd * 1e3, 1), "achieved": round(fld / (msd * 1e-3) / 1e12, 2),
                     "frac": round(fld / (msd * 1e-3) / 1e12 / peak, 4),
                     "single_stream_avg_us": round(per[dom_situ][2] / per[dom_situ][0] * 1e3, 1) if dom_situ in per
                     else None}
    # the north-star kernel set: one train-mode G1+G2 forward (770.95 GFLOP at bs=32, 256^2), HIP events;
    # in the bench dtype and in the other one (the reference computes in fp32)
    flops = gen_fwd_flops(3, 1, args.ngf, B, s, s) + gen_fwd_flops(4, 3, args.ngf, B, s, s)

    def fwd_ms_of():
        with torch.no_grad():
            mp = tr.G1(x)
            tr.G2([x, mp])
            reps = 3
            st = torch.cuda.current_stream()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(st)
            for _ in range(reps):
                mp = tr.G1(x)
                tr.G2([x, mp])
            ev1.record(st)
            ev1.synchronize()
            return ev0.elapsed_time(ev1) / reps

    fwd_ms = fwd_ms_of()
    set_tf = flops / (fwd_ms * 1e-3) / 1e12
    other = "fp32" if args.dtype == "bf16" else "bf16"
    for g in (tr.G1, tr.G2):
        g.set_compute_dtype(other)
    fwd_ms_o = fwd_ms_of()
    for g in (tr.G1, tr.G2):
        g.set_compute_dtype(args.dtype)
    set_tf_o = flops / (fwd_ms_o * 1e-3) / 1e12
    top = sorted(per.items(), key=lambda kv: -kv[1][2])[:10]
    # HBM traffic per launch of the dominant kernel: rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; gfx950
    # FETCH_SIZE x2 correction) over the bench command, committed under profiles/<round>/pmc_traffic.json
    # (this round's profile: profiles/<round>/pmc_traffic.json, made by scripts/profile_round.sh from the bench
    # command itself; the newest round that profiled this kernel)
    traffic, traffic_src, mfma_busy = None, None, None
    import glob
    for fpath in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_traffic.json")), reverse=True):
        try:
            tab = json.load(open(fpath))
        except (OSError, ValueError):
            continue
        hit = [v for k, v in tab.items() if dom in k]
        if hit and args.dtype == "bf16":
            traffic = int(hit[0]["hbm_bytes_per_launch"])
            mfma_busy = hit[0].get("mfma_busy")
            traffic_src = (f"{os.path.relpath(fpath, ROOT)} (round {os.path.basename(os.path.dirname(fpath))}; mean "
                           f"over {hit[0]['launches']} launches of the bench command, all shapes)")
            break
    alg_per_launch = by_dom / n_dom
    conv_ms = sum(v[2] for v in per.values())
    conv_gf = sum(v[1] for v in per.values()) / 1e9
    incl = None  # the dominant kernel with its split-pixel reduction charged to it (weight gradients)
    if dom in whole_single:
        a_incl = fl_dom / (whole_single[dom] * 1e-3) / 1e12
        incl = {"achieved": round(a_incl, 2), "frac": round(a_incl / peak, 4), "ms": round(whole_single[dom], 3),
                "note": "HIP events around each whole stc_conv_wgrad_ex call of this kernel (main kernel + the "
                        "fixed-order split reduction), single-stream step"}
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            # the north-star number (BASELINE.json: >= 40 % of the MFMA roofline on the G1+G2 fused conv forward)
            # beside the dominant kernel's
            "g1g2_forward_frac": round(set_tf / peak, 4),
            "with_reduction": incl,
            "traffic": traffic, "traffic_unit": "bytes/launch",
            "traffic_src": traffic_src,
            "algorithmic_bytes_per_launch": int(alg_per_launch),
            "traffic_over_algorithmic": round(traffic / alg_per_launch, 3) if traffic else None,
            "mfma_busy": mfma_busy,
            "dominant_in_situ": situ_dominant,
            "frac_mode": "single-stream step (each launch alone); frac_in_situ: the same kernel in the bench's "
                         "overlapped step (side-stream networks and weight gradients on)",
            "achieved_in_situ": round(achieved_situ, 2), "frac_in_situ": round(achieved_situ / peak, 4),
            "kernel": f"{dom}: {n_dom} launches in one train step, {fl_dom / 1e9:.2f} GFLOP, {ms_dom:.3f} ms, "
                      f"avg {ms_dom / n_dom * 1e3:.1f} us/launch single-stream, {ms_s / max(n_s, 1) * 1e3:.1f} us "
                      f"in situ (HIP events around the main kernel)",
            "dominant_launches_us": shapes[dom][:40],
            "per_kernel": {k: {"launches": v[0], "gflop": round(v[1] / 1e9, 2), "ms": round(v[2], 3),
                               "alg_mb_per_launch": round(v[3] / v[0] / 1e6, 2),
                               "avg_us": round(v[2] / v[0] * 1e3, 1),
                               "tflops": round(v[1] / (v[2] * 1e-3) / 1e12, 2)} for k, v in top},
            "gemm_kernels_all": {"launches": len(launches), "gflop": round(conv_gf, 2), "ms": round(conv_ms, 3),
                                 "frac": round(conv_gf / conv_ms / peak, 4)},
            "g1g2_forward": {"gflop": round(flops / 1e9, 2), "ms": round(fwd_ms, 3), "tflops": round(set_tf, 2),
                             "frac": round(set_tf / peak, 4), "dtype": args.dtype},
            f"g1g2_forward_{other}": {"gflop": round(flops / 1e9, 2), "ms": round(fwd_ms_o, 3),
                                      "tflops": round(set_tf_o, 2), "frac": round(set_tf_o / PEAK_TFLOPS[other], 4),
                                      "dtype": other}}


def g2_parity(args, local):
    """The metric's 'G2 max-abs vs CPU': G1 -> G2 (train-mode BN, fixture weights with BN gamma ~ 1 so
    the outputs span the tanh range) at ngf=64, 256x256, bs=1 on this GPU vs the CPU oracle."""
    import torch
    from oracle import stcgan_ref as ref
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from fixture_init import fixture_state, uniform
    from stcgan_amd import networks
    dev = torch.device("cuda", local)
    s1 = fixture_state(ref.generator_state_template(3, 1, args.ngf), 11, "one")
    s2 = fixture_state(ref.generator_state_template(4, 3, args.ngf), 12, "one")
    x = uniform((1, 3, args.size, args.size), 311)
    with torch.no_grad():
        mr = ref.generator_forward({k: v.clone() for k, v in s1.items()}, x, True)
        yr = ref.generator_forward({k: v.clone() for k, v in s2.items()}, torch.cat((x, mr), 1), True)
    out = {"config": f"G1->G2 train-mode forward, ngf={args.ngf}, 1x{args.size}x{args.size}, fixture weights"}
    for dt in ("fp32", "bf16"):
        g1 = networks.get_generator(3, 1, ngf=args.ngf)
        g2 = networks.get_generator(4, 3, ngf=args.ngf)
        g1.load_state_dict(s1)
        g2.load_state_dict(s2)
        g1.to(dev).set_compute_dtype(dt).train()
        g2.to(dev).set_compute_dtype(dt).train()
        with torch.no_grad():
            xd = x.to(dev)
            m = g1(xd)
            y = g2([xd, m])
        out[f"g2_maxabs_{dt}"] = float((y.cpu() - yr).abs().max())
        out[f"g1_maxabs_{dt}"] = float((m.cpu() - mr).abs().max())
    out["tolerance_fp32"] = 1e-4
    out["pass_fp32"] = out["g2_maxabs_fp32"] <= 1e-4
    return out


def other_configs(args, local):
    """C2: G1+G2 forward+backward with the L1 data losses, bs=16, fp32 (parity mode); C5: 480x640
    G1->G2 eval-mode inference, bs=8, in the bench dtype; C3 in fp32: the full train step at the bench
    batch computed at the reference's precision.  images/s, HIP events, random init."""
    import torch
    from stcgan_amd import loss, networks
    dev = torch.device("cuda", local)
    res = {}
    g1 = networks.get_generator(3, 1, ngf=args.ngf)
    g2 = networks.get_generator(4, 3, ngf=args.ngf)
    g1.apply(networks.weights_init)
    g2.apply(networks.weights_init)
    g1.to(dev).set_compute_dtype("fp32").train()
    g2.to(dev).set_compute_dtype("fp32").train()
    gen = torch.Generator(device=dev)
    gen.manual_seed(77)
    x = torch.rand((16, 3, 256, 256), generator=gen, device=dev) * 2 - 1
    m = (torch.rand((16, 1, 256, 256), generator=gen, device=dev) < 0.5).float() * 2 - 1
    y = torch.rand((16, 3, 256, 256), generator=gen, device=dev) * 2 - 1
    l1 = loss.DataLoss()

    def c2_step():
        for p in list(g1.parameters()) + list(g2.parameters()):
            p.grad = None
        mp = g1(x)
        yp = g2([x, mp])
        (l1(mp, m) + 5 * l1(yp, y)).backward()

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / reps

    ms = timed(c2_step, 5)
    res["C2_g1g2_fwd_bwd_bs16_fp32"] = {"images_per_s": round(16 / (ms * 1e-3), 2), "ms_per_iter": round(ms, 3),
                                         "tflops": round(72.18e9 * 16 / (ms * 1e-3) / 1e12, 2),
                                         "frac_fp32_mfma": round(72.18e9 * 16 / (ms * 1e-3) / 1e12 / 157.3, 4)}
    g1.set_compute_dtype(args.dtype).eval()
    g2.set_compute_dtype(args.dtype).eval()
    x5 = torch.rand((8, 3, 480, 640), generator=gen, device=dev) * 2 - 1

    def c5():
        with torch.no_grad():
            mp = g1(x5)
            g2([x5, mp])

    ms = timed(c5, 5)
    res[f"C5_infer_480x640_bs8_{args.dtype}"] = {"images_per_s": round(8 / (ms * 1e-3), 2),
                                                  "ms_per_iter": round(ms, 3),
                                                  "tflops": round(113.29e9 * 8 / (ms * 1e-3) / 1e12, 2)}
    del g1, g2
    torch.cuda.empty_cache()
    # C3 at the reference's own precision: the full train step (bench workload, bs=32) computed in fp32
    tr = make_trainer(args.ngf, "fp32", local)
    for net in (tr.G1, tr.G2, tr.D1, tr.D2):
        net.train()
    B = args.batch
    x3 = torch.rand((B, 3, 256, 256), generator=gen, device=dev) * 2 - 1
    m3 = (torch.rand((B, 1, 256, 256), generator=gen, device=dev) < 0.5).float() * 2 - 1
    y3 = torch.rand((B, 3, 256, 256), generator=gen, device=dev) * 2 - 1
    tr.train_step(x3, m3, y3)
    ms = timed(lambda: tr.train_step(x3, m3, y3), 3)
    res[f"C3_train_step_bs{B}_fp32"] = {"images_per_s": round(B / (ms * 1e-3), 2), "ms_per_step": round(ms, 3),
                                        "tflops": round(STEP_GFLOP_PER_IMG * B / (ms * 1e-3) / 1e3, 2),
                                        "frac_fp32_mfma": round(STEP_GFLOP_PER_IMG * B / (ms * 1e-3) / 1e3
                                                                / PEAK_TFLOPS["fp32"], 4)}
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # STC_DIST_BACKEND=gloo: rehearse the multi-rank path on fewer GPUs than ranks
    backend = os.environ.get("STC_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()  # does not initialise the GPU
    local = local % max(ndev, 1) if backend != "nccl" else local
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    # one initialisation (rank 0's weights are broadcast to every rank in STCGAN.__init__); each rank
    # draws its own synthetic shard
    torch.manual_seed(1234)
    tr = make_trainer(args.ngf, args.dtype, local)
    dev = torch.device("cuda", local)
    B, s = args.batch, args.size
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    x = torch.rand((B, 3, s, s), generator=g, device=dev) * 2 - 1
    m = (torch.rand((B, 1, s, s), generator=g, device=dev) < 0.5).float() * 2 - 1
    y = torch.rand((B, 3, s, s), generator=g, device=dev) * 2 - 1
    for net in (tr.G1, tr.G2, tr.D1, tr.D2):
        net.train()

    if args.no_lanes:
        tr.streams = False
    step, mode = (lambda: tr.train_step(x, m, y)), "eager" + ("-nolanes" if args.no_lanes else "")
    if args.graph:
        try:  # (a capture failure, e.g. a backend that cannot be captured, falls back to eager steps)
            step, mode = tr.capture(x, m, y, warmup=1), "hip-graph" + ("-nolanes" if args.no_lanes else "")
        except Exception as e:  # noqa: BLE001
            print(f"bench: graph capture failed ({type(e).__name__}: {e}); eager steps", file=sys.stderr)
            torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    ms_per_step = elapsed / args.steps * 1e3
    value = world * B * args.steps / elapsed

    roofline = roofline_of_step(tr, x, m, y, args, B, s)
    step_gf = (STEP_GFLOP_PER_IMG - SKIPPED_LOGITS_GFLOP_PER_IMG) * B
    step_tf = step_gf / (ms_per_step * 1e-3) / 1e3
    roofline["whole_step"] = {"gflop": round(step_gf, 1), "ms": round(ms_per_step, 3),
                              "tflops": round(step_tf, 2), "frac": round(step_tf / PEAK_TFLOPS[args.dtype], 4),
                              "note": "algorithmic conv FLOPs of the step as run: the two G-step real-input "
                                      "discriminator calls skip their logits conv with loss type normal (its output "
                                      "is unused; engine stats_only), 2 x 0.47 GF at bs 32, not counted"}
    roofline["whole_step_frac"] = roofline["whole_step"]["frac"]
    if world > 1:
        dist.barrier()

    extras, cpu = {}, None
    if rank == 0 and world == 1 and not args.no_extras:
        del tr
        torch.cuda.empty_cache()
        extras["parity"] = g2_parity(args, local)
        extras["configs"] = other_configs(args, local)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
    if rank == 0:
        out = {"metric": METRIC, "value": round(value, 3), "unit": "images/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
               "data": "synthetic (x,y~U(-1,1), m=+-1; reference weights_init)",
               "config": {"workload": "full ST-CGAN train step (G1,G2,D1,D2 fwd/bwd + MSE-cGAN/L1 + Adam), "
                                      f"{s}x{s}", "global_batch": B * world, "per_gpu_batch": B,
                          "image_size": s, "ngf": args.ngf, "parallelism": f"dp{world}", "step_launch": mode},
               "roofline": roofline, "cpu_baseline": cpu, **extras}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
