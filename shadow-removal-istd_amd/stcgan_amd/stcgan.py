"""Drop-in replacement for the STCGAN trainer (STCGAN/stcgan.py:25-433) on MI355X.

Public surface kept: ``STCGAN(args)``, ``train(epochs)``, ``run_epoch(training)``,
``infer()``, ``save(weights, suffix)``, ``init_weight(...)``, the G1/G2/D1/D2,
optim_G/optim_D, decay_G/decay_D, adv_loss/data_loss attributes, the losses
dict returned by run_epoch and the ``{G1,G2,D1,D2}-{suffix}.pt`` checkpoints.

Differences that do not change results:
  * the per-iteration ``.item()`` / ``.cpu()`` syncs of the reference
    (STCGAN/stcgan.py:256-262, 308-312) are replaced by on-device accumulators
    read once per epoch;
  * the input concatenations of the discriminators/generator are passed as
    source lists (zero-copy: the first layer gathers the channels itself);
  * multi-GPU is one process per GPU with an RCCL gradient all-reduce
    (parallel.py) instead of nn.DataParallel.
Loaders: any iterable of (names, x, m, y) batches; with ``args.data_dir`` and no
loader passed, the reference's two ISTD loaders (STCGAN/stcgan.py:73-104) are built
on data.ISTDLoader (decode on the host, Resize / RandomScale / RandomRotate / flip /
crop on the device), each rank taking its shard of the global ``args.batch_size``.
"""
import contextlib
import datetime
import logging
import os
import time

import numpy as np
import torch
import torch.nn as nn

from . import engine
from . import ops
from . import networks
from . import parallel
from .loss import AdversarialLoss, DataLoss, d_objective, d_term_grad, g_objective
from .optim import Adam


class SyntheticTriplets:
    """Synthetic ISTD-shaped batches (x, y ~ U(-1,1), m = +-1), generated on the device."""

    def __init__(self, n_batches, batch_size, size=256, seed=1234, device="cuda"):
        self.n, self.bs, self.size, self.seed, self.device = n_batches, batch_size, size, seed, device

    def __len__(self):
        return self.n

    def __iter__(self):
        g = torch.Generator(device=self.device)
        g.manual_seed(self.seed)
        s = self.size
        for i in range(self.n):
            x = torch.rand((self.bs, 3, s, s), generator=g, device=self.device) * 2 - 1
            m = (torch.rand((self.bs, 1, s, s), generator=g, device=self.device) < 0.5).float() * 2 - 1
            y = torch.rand((self.bs, 3, s, s), generator=g, device=self.device) * 2 - 1
            yield ([f"synthetic_{i}_{j}" for j in range(self.bs)], x, m, y)


def batch_weight(local_n, global_n, world):
    """Weight of one rank's batch means in the rank average (parallel.average_scalars): n_local * world /
    n_global, so that the average of the weighted per-rank means is the mean over the global batch -- what the
    reference computes on DataParallel's gathered outputs -- also for a ragged final batch, whose shards differ
    by one sample (data.shard_bounds).  1.0 at world size 1 or when the global size is unknown."""
    if world <= 1 or not global_n:
        return 1.0
    return local_n * world / global_n


def weighted_loss(loss, weight):
    """The loss a rank back-propagates: its shard mean scaled by ``weight`` (batch_weight).  The gradient
    exchange averages the ranks' gradients with equal weight, so sum_r w_r * grad(mean over shard r) / world =
    grad(mean over the global batch) -- DataParallel's gradient, whose loss is computed on the gathered outputs
    (STCGAN/stcgan.py:53-59) -- also when a ragged final batch gives the ranks shards of different sizes."""
    return loss if weight == 1.0 else loss * weight


def accumulate(acc, vals, d_out, weight=1.0):
    """Add one step's losses (``vals``: device fp32 scalars) and mean discriminator outputs (``d_out``: C1_real,
    C1_fake, C2_real, C2_fake) into the float64 device sums ``acc``, each value widened to float64 first (the
    reference adds the float32 results' .item() to Python floats) and scaled by ``weight`` (batch_weight)."""
    for k, v in vals.items():
        acc[k] = acc[k] + v.double() * weight
    for k, c in zip(("D1_real", "D1_fake", "D2_real", "D2_fake"), d_out):
        acc[k] = acc[k] + c.mean().double() * weight


# loss type "normal": the G step's statistics-only real-input discriminator calls after the fake-input ones (their
# running-statistics updates applied in the reference's order); False (A/B, tests): before them, as the reference
LATE_STATS_CALLS = True
# loss type "normal": each discriminator call's D-step backward right after its forward (STCGAN._term_backward):
# 1 = the real-input calls', 2 = every call's; 0 (A/B, tests): one D-objective backward after the fake forwards, as
# the reference does
EARLY_D_BACKWARD = 2

class STCGAN(object):

    def __init__(self, args, train_loader=None, valid_loader=None):
        self.logger = logging.getLogger(__name__)
        if not torch.cuda.is_available():
            raise RuntimeError("stcgan_amd.STCGAN needs a ROCm GPU")
        self.device = torch.device(self._device_of(args))
        ngf = getattr(args, "ngf", 64)
        self.G1 = networks.get_generator(in_channels=3, out_channels=1, ngf=ngf)
        self.G2 = networks.get_generator(in_channels=3 + 1, out_channels=3, ngf=ngf)
        self.D1 = networks.get_discriminator(in_channels=3 + 1, ndf=ngf, n_layers=3, use_sigmoid=False)
        self.D2 = networks.get_discriminator(in_channels=3 + 3 + 1, ndf=ngf, n_layers=3, use_sigmoid=False)
        tasks = getattr(args, "tasks", ["train"])
        if "infer" in tasks and "train" not in tasks:
            assert args.load_weights_g1 is not None
            assert args.load_weights_g2 is not None
        self.init_weight(g1_weights=getattr(args, "load_weights_g1", None),
                         g2_weights=getattr(args, "load_weights_g2", None),
                         d1_weights=getattr(args, "load_weights_d1", None),
                         d2_weights=getattr(args, "load_weights_d2", None))
        dtype = getattr(args, "dtype", "fp32")
        for net in (self.G1, self.G2, self.D1, self.D2):
            net.to(self.device)
            net.set_compute_dtype(dtype)
        # every rank starts from rank 0's weights (DataParallel replicates dev0's module)
        parallel.broadcast_state([self.G1, self.G2, self.D1, self.D2])
        self.start_epoch = 0
        self.optim_G = Adam(list(self.G1.parameters()) + list(self.G2.parameters()),
                            lr=args.lr_G, betas=(args.beta1, args.beta2))
        self.optim_D = Adam(list(self.D1.parameters()) + list(self.D2.parameters()),
                            lr=args.lr_D, betas=(args.beta1, args.beta2))
        self.decay_G = torch.optim.lr_scheduler.ReduceLROnPlateau(self.optim_G, cooldown=10, min_lr=1e-7, factor=0.8)
        self.decay_D = torch.optim.lr_scheduler.ReduceLROnPlateau(self.optim_D, cooldown=10, min_lr=1e-7, factor=0.8)
        # each network's gradients live in one flat buffer (parallel.FlatGrads), cut into buckets that the
        # engine reports complete while the backward runs (parallel.BucketExchange): with data parallelism each
        # bucket is averaged over the ranks (RCCL) right then.  overlap_optim: the optimiser also updates each
        # bucket right after (optim.Adam.overlap) -- bit-identical.  On by default with data parallelism: the
        # update of the early buckets then runs while the last ones are still being exchanged, so the G step's
        # tail after its backward is the last bucket's all-reduce + its update, not the whole exchange + the whole
        # update (scripts/exchange_timeline.py).  Off at world 1, where there is nothing to hide: the updates' HBM
        # traffic only moved time into the backward's kernels (round-3 A/B, scripts/ab_overlap.py: 13.22 vs 13.05
        # ms/step).
        world = parallel.world()
        self.bucket_mb = float(getattr(args, "bucket_mb", 16 if world > 1 else 8))
        for net in (self.G1, self.G2, self.D1, self.D2):
            net.grad_exchange = parallel.BucketExchange(parallel.flat_grads(net), self.bucket_mb)
        self.set_overlap_optim(bool(getattr(args, "overlap_optim", world > 1)))
        # discriminators on side HIP streams (train_step / _lanes); off for a strictly serial step
        self.streams = bool(getattr(args, "streams", True))
        self.lane_carry = bool(getattr(args, "lane_carry", True))
        self._lane_inputs = None
        self._lanes_stale = True  # the side lanes must wait for the main stream before their next work
        # loss type "normal": the D and G objectives as one fused node each (loss.d_objective / g_objective)
        self.fused_objectives = bool(getattr(args, "fused_objectives", True))
        self._gout_one = {}  # stream handle -> fp32 1 made on that stream (_term_backward)
        self._side = None

        data_dir = getattr(args, "data_dir", None)
        if data_dir is not None and train_loader is None and valid_loader is None:
            train_loader, valid_loader = self.istd_loaders(args)
        self.train_loader = train_loader
        self.valid_loader = valid_loader

        if "train" in tasks:
            self.d_loss_fn = getattr(args, "D_loss_fn", "standard")
            self.d_loss_type = getattr(args, "D_loss_type", "normal")
            # the reference compares against the misspelt "leastsqure" (STCGAN/stcgan.py:111-112):
            # ls is therefore always False -> MSE with labels 1/0.  Kept as is.
            self.adv_loss = AdversarialLoss(ls=(self.d_loss_fn == "leastsqure"))
            self.adv_loss.to(self.device)
            self.data_loss = DataLoss().to(self.device)
            self.lambda1 = 5     # data2 loss
            self.lambda2 = 0.1   # CGAN1 loss
            self.lambda3 = 0.1   # CGAN2 loss
            self.adapt = getattr(args, "softadapt", False)
            self.weights_dir = getattr(args, "weights", None)
            self.log_interval = getattr(args, "log_every", 3)
            self.valid_interval = getattr(args, "valid_every", 10)
        if "infer" in tasks:
            self.inferd_dir = getattr(args, "infered", None)

    def set_overlap_optim(self, on):
        """Update each gradient bucket as the backward completes it (optim.Adam.overlap) or after the backward."""
        self.overlap_optim = bool(on)
        self.optim_G.overlap([self.G1.grad_exchange, self.G2.grad_exchange], on=self.overlap_optim)
        self.optim_D.overlap([self.D1.grad_exchange, self.D2.grad_exchange], on=self.overlap_optim)

    @staticmethod
    def _device_of(args):
        """The reference trains on ``args.devices`` with nn.DataParallel (STCGAN/stcgan.py:53-59).  Here
        data parallelism is one process per GPU: each rank takes ``devices[local rank]``.  A multi-device
        list in a single process cannot be honoured silently, so it is an error."""
        devs = list(getattr(args, "devices", None) or ["cuda"])
        w = parallel.world()
        if len(devs) > 1 and w == 1:
            raise RuntimeError(
                f"stcgan_amd: args.devices lists {len(devs)} devices, but data parallelism runs one process per "
                f"GPU: launch the script with `torchrun --nproc-per-node {len(devs)} ...` (each rank uses "
                f"devices[LOCAL_RANK] and the gradients are all-reduced over RCCL), or pass one device")
        if w > 1:
            local = int(os.environ.get("LOCAL_RANK", parallel.rank()))
            return devs[local] if len(devs) >= w else f"cuda:{local % max(torch.cuda.device_count(), 1)}"
        return devs[0]

    def _exchange(self, names, expected):
        """Set how many backward calls write each network's gradients in this step (the discriminators are
        called on real and on fake inputs inside the D step's graph)."""
        for n in names:
            ex = parallel.exchange_of(getattr(self, n))
            if ex is not None:
                ex.expected = expected

    def _finish_exchange(self, names):
        for n in names:
            ex = parallel.exchange_of(getattr(self, n))
            if ex is not None:
                ex.finish()

    def istd_loaders(self, args):
        """The reference's train/valid loaders (STCGAN/stcgan.py:73-104) on data.ISTDLoader."""
        from .data import ISTDLoader
        self.logger.info("Creating data loaders")
        common = dict(batch_size=args.batch_size, datas=("img", "mask", "target"),
                      workers=getattr(args, "workers", 0), rank=parallel.rank(), world=parallel.world(),
                      device=self.device)
        train = ISTDLoader(args.data_dir, "train", resize=(300, 400), scale=getattr(args, "aug_scale", 0.05),
                           angle=getattr(args, "aug_angle", 15), flip_prob=0.5,
                           crop_size=getattr(args, "image_size", 256), shuffle=True, drop_last=True, **common)
        valid = ISTDLoader(args.data_dir, "test", resize=(256, 256), shuffle=False, drop_last=False, **common)
        return train, valid

    # ------------------------------------------------------------------ training
    def train(self, epochs=5000):
        self.logger.info("Start training")
        best_loss = 100000.0
        start_time = time.time()
        for epoch in range(self.start_epoch, epochs):
            measures = self.run_epoch()
            if epoch % self.log_interval == 0:
                self.logger.info(f"epoch {epoch}: {measures['Loss']}")
                if self.weights_dir:
                    self.save(self.weights_dir, "latest")
            if epoch % self.valid_interval == 0 and self.valid_loader is not None:
                measures = self.run_epoch(training=False)
                if measures["Loss"]["total"] < best_loss:
                    best_loss = measures["Loss"]["total"]
                    if self.weights_dir:
                        self.save(self.weights_dir, "best")
                    self.logger.info(f"Improvement after epoch {epoch}, error = {best_loss:4f}")
        total_time = datetime.timedelta(seconds=(time.time() - start_time))
        self.logger.info(f"Training time {total_time}")
        self.logger.info(f"Best validation loss: {best_loss:.3f}")

    def _d_losses(self, C1_real, C1_fake, C2_real, C2_fake):
        adv = self.adv_loss
        t = self.d_loss_type
        mean0 = parallel.global_mean0  # C.mean(dim=0) over the global batch (DataParallel gathers)
        if t == "normal":
            D1_loss = (adv(C1_fake, is_real=False) + adv(C1_real, is_real=True)) * 0.5
            D2_loss = (adv(C2_fake, is_real=False) + adv(C2_real, is_real=True)) * 0.5
        elif t == "rel":
            D1_loss = adv(C1_real - C1_fake, is_real=True)
            D2_loss = adv(C2_real - C2_fake, is_real=True)
        else:  # "rel_avg"
            D1_loss = (adv(C1_fake - mean0(C1_real), is_real=False)
                       + adv(C1_real - mean0(C1_fake), is_real=True)) * 0.5
            D2_loss = (adv(C2_fake - mean0(C2_real), is_real=False)
                       + adv(C2_real - mean0(C2_fake), is_real=True)) * 0.5
        return D1_loss, D2_loss

    def _g_losses(self, C1_real, C1_fake, C2_real, C2_fake):
        adv = self.adv_loss
        t = self.d_loss_type
        if t == "normal":
            return adv(C1_fake, is_real=True), adv(C2_fake, is_real=True)
        if t == "rel":
            return adv(C1_fake - C1_real, is_real=True), adv(C2_fake - C2_real, is_real=True)
        mean0 = parallel.global_mean0
        G1_loss = (adv(C1_fake - mean0(C1_real), is_real=True)
                   + adv(C1_real - mean0(C1_fake), is_real=False)) * 0.5
        # as the reference: the rel_avg G2 loss is computed from the D1 outputs (STCGAN/stcgan.py:286-290)
        G2_loss = (adv(C1_fake - mean0(C1_real), is_real=True)
                   + adv(C1_real - mean0(C1_fake), is_real=False)) * 0.5
        return G1_loss, G2_loss

    def _lanes(self):
        """(main, D1 lane, D2 lane): the discriminators run on their own HIP streams so their
        kernels overlap the generators' (and each other's) -- many of the step's launches are
        latency-bound small grids that leave most of the 256 CUs idle.  Autograd runs each
        network's backward on the stream its forward ran on and inserts the cross-stream
        waits for the gradients that flow between them."""
        main = torch.cuda.current_stream(self.device)
        if not self.streams:
            return main, None, None
        if getattr(self, "_side", None) is None:
            self._side = (torch.cuda.Stream(self.device), torch.cuda.Stream(self.device))
        return (main,) + self._side

    def _on(self, lane, net, srcs, after=None):
        """net(srcs) on ``lane`` (None = the current stream), after the main-stream event ``after``.
        (A lane output read by several main-stream ops gets its gradients summed by autograd; that sum is
        safe across streams on this torch: tests/test_gpu_stream_hazards.py.)"""
        if lane is None:
            return net(srcs)
        with torch.cuda.stream(lane):
            if after is not None:
                lane.wait_event(after)
            for s in srcs:
                s.record_stream(lane)
            out = net(srcs)
        out.record_stream(torch.cuda.current_stream(self.device))
        return out

    def _term_backward(self, lane, C, lam, weight, real):
        """Back-propagate one term of the D objective (loss type normal) from its logits (on its lane)."""
        with (torch.cuda.stream(lane) if lane is not None else contextlib.nullcontext()):
            if weight == 1.0:  # (the objective's incoming gradient: one fp32 1, made once per stream that reads it)
                key = lane.cuda_stream if lane is not None else None
                gout = self._gout_one.get(key)
                if gout is None:
                    gout = self._gout_one[key] = torch.ones((), dtype=torch.float32, device=self.device)
            else:  # (weighted_loss: loss * weight, whose backward hands the objective fp32(weight))
                gout = torch.full((), weight, dtype=torch.float32, device=self.device)
            torch.autograd.backward(C, d_term_grad(self.adv_loss, C, lam, gout, real))

    def train_step(self, x, m, y, training=True, acc=None, inputs_ready=None, weight=1.0):
        """One iteration of STCGAN.run_epoch (STCGAN/stcgan.py:208-312): D step then G step.
        Returns the on-device loss scalars (no host sync).  The call order of every network
        (and so every BN running-statistics update) is the reference's; with ``streams`` the
        discriminator calls run on side streams (see _lanes) -- same kernels, same results."""
        self.optim_D.zero_grad()
        self.optim_G.zero_grad()
        main, l1, l2 = self._lanes()
        if l1 is None and inputs_ready is not None:
            main.wait_event(inputs_ready)
        if l1 is not None:
            # The side lanes start with the discriminators' real-input forwards, which need the D weights of
            # the last D update (the lanes waited for it before the previous G step) and the inputs.  With the
            # inputs of the previous step (same tensors, unmodified) they need nothing else from the main
            # stream and overlap its G backward and G update; new inputs were produced on the main stream.
            # Lane-allocated tensors read on the main stream are record_stream'ed (outputs, input gradients).
            # inputs_ready: an event after which x, m, y are complete (produced on another stream, not read
            # by anything but this step), e.g. run_epoch's input stream
            # the previous step's inputs are held (not an id/address key: both are reused once a tensor dies)
            same = (self._lane_inputs is not None
                    and all(a is b and a._version == v for a, b, v in zip((x, m, y), *self._lane_inputs)))
            if inputs_ready is not None:
                for t in (x, m, y):
                    t.record_stream(main)
                main.wait_event(inputs_ready)
            if self._lanes_stale or not self.lane_carry:
                # D state written on the main stream outside the step (construction, broadcasts, checkpoint
                # loads, a validation pass): the lanes start after it
                engine.wait_stream(l1, main)
                engine.wait_stream(l2, main)
                self._lanes_stale = False
            elif inputs_ready is not None:
                l1.wait_event(inputs_ready)
                l2.wait_event(inputs_ready)
            elif not same:
                engine.wait_stream(l1, main)
                engine.wait_stream(l2, main)
            self._lane_inputs = ((x, m, y), tuple(t._version for t in (x, m, y)))
            self.D1.grad_consumer = self.D2.grad_consumer = main
        # each discriminator sees the same real and fake inputs in the D and the G step: gather them once
        self.D1.input_cache, self.D2.input_cache = {}, {}
        try:
            return self._step(x, m, y, training, acc, main, l1, l2, weight)
        finally:
            self.D1.input_cache = self.D2.input_cache = None

    def _step(self, x, m, y, training, acc, main, l1, l2, weight=1.0):
        with torch.set_grad_enabled(training):
            self.optim_D.zero_grad()
            self.D1.requires_grad_(True)
            self.D2.requires_grad_(True)
            # loss type "normal": each discriminator call's backward runs right after its forward (each term of the
            # objective involves one logits tensor, loss.d_term_grad) -- the real-input ones off the D step's
            # critical path, overlapping the generators' forwards (and, carried over on the lanes, the previous
            # step's G update), D1's fake-input one overlapping G2's forward; the objective below then takes the
            # logits detached.  The D gradients' real + fake sum is the same fp32 addition: bit-identical.
            early = training and EARLY_D_BACKWARD and self.d_loss_type == "normal" and self.fused_objectives
            if early:
                self._exchange(("D1", "D2"), 2)  # real + fake calls
            C1_real = self._on(l1, self.D1, [x, m])
            if early:
                self._term_backward(l1, C1_real, self.lambda2, weight, True)
            C2_real = self._on(l2, self.D2, [x, m, y])
            if early:
                self._term_backward(l2, C2_real, self.lambda3, weight, True)
            m_pred = self.G1(x)
            ev_m = engine.hold(main.record_event()) if l1 is not None else None
            C1_fake = self._on(l1, self.D1, [x, m_pred.detach()], after=ev_m)
            y_pred = self.G2([x, m_pred])
            ev_y = engine.hold(main.record_event()) if l1 is not None else None
            if early and EARLY_D_BACKWARD > 1:
                self._term_backward(l1, C1_fake, self.lambda2, weight, False)
            C2_fake = self._on(l2, self.D2, [x, m_pred.detach(), y_pred.detach()], after=ev_y)
            if early and EARLY_D_BACKWARD > 1:
                self._term_backward(l2, C2_fake, self.lambda3, weight, False)
            if l1 is not None:
                engine.wait_stream(main, l1)
                engine.wait_stream(main, l2)
            if self.d_loss_type == "normal" and self.fused_objectives:  # one node (loss.d_objective)
                full = early and EARLY_D_BACKWARD > 1  # (every term back-propagated above: values only here)
                D_loss, D1_loss, D2_loss = d_objective(self.adv_loss, C1_fake.detach() if full else C1_fake,
                                                       C1_real.detach() if early else C1_real,
                                                       C2_fake.detach() if full else C2_fake,
                                                       C2_real.detach() if early else C2_real,
                                                       self.lambda2, self.lambda3)
            else:
                D1_loss, D2_loss = self._d_losses(C1_real, C1_fake, C2_real, C2_fake)
                D_loss = self.lambda2 * D1_loss + self.lambda3 * D2_loss
            if training:
                if not early:
                    self._exchange(("D1", "D2"), 2)  # real + fake calls
                if not (early and EARLY_D_BACKWARD > 1):
                    weighted_loss(D_loss, weight).backward()
                self._finish_exchange(("D2", "D1"))
                self.optim_D.step()
            d_out = (C1_real.detach(), C1_fake.detach(), C2_real.detach(), C2_fake.detach())

            self.optim_G.zero_grad()
            self.D1.requires_grad_(False)
            self.D2.requires_grad_(False)
            if training:  # D is not updated when validating
                if l1 is not None:  # after optim_D.step
                    engine.wait_stream(l1, main)
                    engine.wait_stream(l2, main)
                # loss type "normal": the G objective does not read C_real; the calls still run (the reference
                # makes them, STCGAN/stcgan.py:269-272) for their BatchNorm running statistics, minus the
                # logits layer (engine: stats_only)
                unused = self.d_loss_type == "normal"
                # ... and, with LATE_STATS_CALLS, after the fake-input calls (whose running-statistics updates are
                # held back and applied after theirs, in the reference's order: real then fake per BatchNorm) -- the
                # G step's critical path (D update -> fake-input forwards -> their input gradients -> G backward)
                # no longer waits for two forwards whose outputs nothing reads
                late = unused and LATE_STATS_CALLS
                if not late:
                    self.D1.stats_only = self.D2.stats_only = unused
                    C1_real = self._on(l1, self.D1, [x, m])
                    C2_real = self._on(l2, self.D2, [x, m, y])
                    self.D1.stats_only = self.D2.stats_only = False
                if unused:  # (zero-element placeholders: the logits were not computed)
                    C1_real = C2_real = None
                if late:
                    held = ([], [])
                    self.D1.defer_running, self.D2.defer_running = held
                try:
                    C1_fake = self._on(l1, self.D1, [x, m_pred])
                    C2_fake = self._on(l2, self.D2, [x, m_pred, y_pred])
                finally:
                    self.D1.defer_running = self.D2.defer_running = None
                if l1 is not None:
                    engine.wait_stream(main, l1)
                    engine.wait_stream(main, l2)
            if self.d_loss_type == "normal" and self.fused_objectives:
                G_loss, G1_loss, G2_loss, data1_loss, data2_loss = g_objective(
                    self.adv_loss, m_pred, m, y_pred, y, C1_fake, C2_fake, self.lambda1, self.lambda2, self.lambda3)
            else:
                G1_loss, G2_loss = self._g_losses(C1_real, C1_fake, C2_real, C2_fake)
                data1_loss = self.data_loss(m_pred, m)
                data2_loss = self.data_loss(y_pred, y)
                G_loss = data1_loss + self.lambda1 * data2_loss + self.lambda2 * G1_loss + self.lambda3 * G2_loss
            if training:
                self._exchange(("G1", "G2"), 1)
                weighted_loss(G_loss, weight).backward()
                if late:  # the statistics-only real-input calls, then the fake calls' held running updates
                    self.D1.stats_only = self.D2.stats_only = True
                    try:
                        self._on(l1, self.D1, [x, m])
                        self._on(l2, self.D2, [x, m, y])
                    finally:
                        self.D1.stats_only = self.D2.stats_only = False
                    for lane, lst in zip((l1, l2), held):
                        with (torch.cuda.stream(lane) if lane is not None else contextlib.nullcontext()):
                            for item in lst:
                                ops.bn_running_update(*item)
                self._finish_exchange(("G2", "G1"))
                self.optim_G.step()
        if l1 is not None:  # nothing on the side lanes outlives the step
            engine.wait_stream(main, l1)
            engine.wait_stream(main, l2)
        vals = dict(D1=D1_loss.detach(), D2=D2_loss.detach(), D=D_loss.detach(), G1=G1_loss.detach(),
                    G2=G2_loss.detach(), data1=data1_loss.detach(), data2=data2_loss.detach(), G=G_loss.detach())
        if acc is not None:
            accumulate(acc, vals, d_out, weight)
        return vals

    def capture(self, x, m, y, warmup=1):
        """train_step(x, m, y) captured as one HIP graph; returns ``replay()``, which runs one more full
        train step (both D and G updates) on whatever x, m, y then hold (refill them in place: the graph
        keeps their addresses).  Kernels, streams and memory are those of the eager step -- the side lanes
        and weight-gradient streams become branches of the graph, every activation lives in the graph's
        private pool -- but the ~700 launches of a step leave the host: one graph launch per step.  The
        optimisers switch to device-resident step counts (optim.Adam.device_step) so that replays advance
        them; their host-side counts are synced by state_dict().  Replay is bit-identical to the eager
        step (tests/test_gpu_graph.py).  World size > 1 needs the RCCL backend (collectives are captured
        too)."""
        import torch.distributed as dist
        if parallel.world() > 1 and dist.get_backend() != "nccl":
            raise RuntimeError("STCGAN.capture: multi-process capture needs the nccl (RCCL) backend")
        main, l1, l2 = self._lanes()
        if l1 is not None:  # (see engine.NO_SIDE_IN_CAPTURE; pooled stream handles recur across trainers)
            if engine.SIDE_IN_CAPTURE:
                engine.NO_SIDE_IN_CAPTURE.difference_update((l1.cuda_stream, l2.cuda_stream))
            else:
                engine.NO_SIDE_IN_CAPTURE.update((l1.cuda_stream, l2.cuda_stream))
        cap = torch.cuda.Stream(self.device)
        engine.wait_stream(cap, main)
        with torch.cuda.stream(cap):
            for _ in range(max(1, warmup)):  # steady state: packed operands, tables, streams, flat gradients
                self.train_step(x, m, y)
            for o in (self.optim_G, self.optim_D):
                o.device_step(True)
            # eager steps in device-step mode until both optimisers run their steady-state path with their
            # device counters created (a packed operand first made in a step -- the discriminators' input-
            # gradient operands appear in the first G step -- sends the next step down the full path)
            for _ in range(2):
                self.train_step(x, m, y)
        engine.wait_stream(main, cap)
        torch.cuda.synchronize(self.device)
        graph = torch.cuda.CUDAGraph()
        self._lanes_stale = True  # inside the capture the lanes must fork from the capturing stream
        engine.CAPTURE_EVENTS = []  # every event recorded / waited in the capture lives until it has ended
        try:
            self._capture_into(graph, cap, x, m, y, l1, l2)
        finally:
            engine.CAPTURE_EVENTS = None
        self._graph = graph
        # the optimisers' device pointer tables the captured launches read: kept alive even when a later eager
        # step on the general path replaces them (freed, their memory could be reused under the graph)
        self._graph_refs = [t for o in (self.optim_G, self.optim_D) for f in o._fast.values()
                            for t in [f["table"]] + [sub[0] for sub in f["subs"].values()]]

        def replay():
            for o in (self.optim_G, self.optim_D):
                o.sync_lr()
            graph.replay()
        return replay

    def _capture_into(self, graph, cap, x, m, y, l1, l2):
        with torch.cuda.graph(graph, stream=cap):
            if l1 is not None and engine.SIDE_IN_CAPTURE:
                # the lanes' weight-gradient side streams join the capture from the capturing stream itself, before
                # their first wait on a lane (a side stream whose first capture edge came from a lane, itself
                # forked from the capturing stream, crashed the capture on this ROCm: scripts/graph_capture_probe.py)
                for ln in (l1, l2):
                    ent = engine._WG_SIDE.get(ln.cuda_stream)
                    if ent is not None:
                        engine.wait_stream(ent[0], cap)
            self.train_step(x, m, y)

    def run_epoch(self, training=True):
        for net in (self.G1, self.G2, self.D1, self.D2):
            net.train(training)
        if not training:  # eval-mode replicas use dev0's running statistics
            parallel.broadcast_buffers([self.G1, self.G2, self.D1, self.D2])
        self._lanes_stale = True  # (the broadcast above, a checkpoint load, a caller's writes between epochs)
        keys = ["G", "D", "D1", "D2", "G1", "G2", "data1", "data2"]
        # float64 sums, as the reference's Python-float accumulation of .item() values (STCGAN/stcgan.py:256-262,
        # 308-312) that ReduceLROnPlateau then reads
        acc = {k: torch.zeros((), dtype=torch.float64, device=self.device)
               for k in keys + ["D1_real", "D1_fake", "D2_real", "D2_fake"]}
        data_loader = self.train_loader if training else self.valid_loader
        n_batches = 0
        # with the side lanes, batches are prepared on an input stream and handed over with an event, so the
        # lanes wait for the batch only (not for the main stream's G backward and update of the last step)
        lanes = self._lanes()[1] is not None
        if lanes and getattr(self, "_in_stream", None) is None:
            self._in_stream = torch.cuda.Stream(self.device)
        it = iter(data_loader)
        while True:
            if lanes:
                with torch.cuda.stream(self._in_stream):
                    b = next(it, None)
                    if b is not None:
                        b = [t.to(self.device, non_blocking=True) for t in b[1:]]
                    ready = self._in_stream.record_event()
            else:
                b = next(it, None)
                if b is not None:
                    b = [t.to(self.device, non_blocking=True) for t in b[1:]]
                ready = None
            if b is None:
                break
            x, m, y = b
            # a ragged final batch is split unevenly over the ranks: weight each rank's means by its share
            w = batch_weight(x.shape[0], getattr(data_loader, "last_global", None), parallel.world())
            self.train_step(x, m, y, training=training, acc=acc, inputs_ready=ready, weight=w)
            n_batches += 1
        # global-batch values on every rank (DataParallel computes the losses on the gathered
        # batch), so each rank's ReduceLROnPlateau sees the same sums: one collective, one host sync
        acc = parallel.average_scalars(acc)
        host = {k: float(v) for k, v in acc.items()}
        loss = {k: host[k] for k in keys}
        if training:
            self.decay_G.step(loss["G"])
            self.decay_D.step(loss["D"])
        loss["total"] = loss["G"] * 0.8 + loss["D"] * 0.2
        n = max(n_batches, 1)
        for k in loss:
            loss[k] /= n
        D1_out = {"real": host["D1_real"] / n, "fake": host["D1_fake"] / n}
        D2_out = {"real": host["D2_real"] / n, "fake": host["D2_fake"] / n}
        return {"Loss": loss, "D1_out": D1_out, "D2_out": D2_out}

    # ------------------------------------------------------------------ inference
    def infer(self, out_size=(256, 192)):
        """G1 -> G2 in eval mode over the validation loader (STCGAN/stcgan.py:332-381), with the
        reference's output stage on the GPU (ops.infer_output: x*0.5+0.5, cv.resize to
        ``out_size`` = (width, height) INTER_LINEAR, float2uint truncation).  Writes
        ``{infered}/mask/<name>.png`` and ``{infered}/shadowless/<name>.png`` (the uint8 arrays
        cv.imwrite receives: mask single-channel, shadowless in the loader's BGR channel order);
        returns the list of (name, mask uint8 [h, w], shadowless uint8 [h, w, 3])."""
        from . import ops
        ow, oh = out_size
        results = []
        with torch.no_grad():
            self.G1.eval()
            self.G2.eval()
            parallel.broadcast_buffers([self.G1, self.G2])
            for (filenames, x, _, _) in self.valid_loader:
                x = x.to(self.device, non_blocking=True)
                m_pred = self.G1(x)
                y_pred = self.G2([x, m_pred])
                m_u8 = ops.infer_output(m_pred, oh, ow).cpu().numpy()
                y_u8 = ops.infer_output(y_pred, oh, ow).cpu().numpy()
                for i, name in enumerate(filenames):
                    mk = m_u8[i, :, :, 0]
                    sl = y_u8[i]
                    results.append((name, mk, sl))
                    if self.inferd_dir:
                        _write_png(os.path.join(self.inferd_dir, "mask", name + ".png"), mk)
                        _write_png(os.path.join(self.inferd_dir, "shadowless", name + ".png"), sl)
        return results

    # ------------------------------------------------------------------ checkpoints
    def save(self, weights=None, suffix="latest"):
        # rank 0's BN running statistics are the reference's dev0 replica statistics
        if parallel.rank() != 0:
            return
        if weights is None:
            weights = self.weights_dir
        os.makedirs(weights, exist_ok=True)
        for name in ("G1", "G2", "D1", "D2"):
            module = getattr(self, name)
            module = module.module if isinstance(module, nn.DataParallel) else module
            torch.save(module.state_dict(), os.path.join(weights, f"{name}-{suffix}.pt"))

    def save_checkpoint(self, epoch, path="./checkpoint.tar"):
        """Full training state (src/cgan.py:494-511): epoch, the four state_dicts, both
        optimisers (Adam moments + step counts) and both LR schedulers; rank 0 only."""
        if parallel.rank() != 0:
            return
        mod = {k: (getattr(self, k).module if isinstance(getattr(self, k), nn.DataParallel) else getattr(self, k))
               for k in ("G1", "G2", "D1", "D2")}
        torch.save({"epoch": epoch, **{k: m.state_dict() for k, m in mod.items()},
                    "optim_G": self.optim_G.state_dict(), "optim_D": self.optim_D.state_dict(),
                    "decay_G": self.decay_G.state_dict(), "decay_D": self.decay_D.state_dict()}, path)

    def load_checkpoint(self, path="./checkpoint.tar"):
        """Resume from save_checkpoint (src/cgan.py:513-523; restores decay_G as well -- the
        reference loads decay_D twice)."""
        ck = torch.load(path, map_location=self.device, weights_only=True)
        self._lanes_stale = True  # the loads below write D state on the main stream
        self.start_epoch = ck["epoch"]
        for k in ("G1", "G2", "D1", "D2"):
            getattr(self, k).load_state_dict(ck[k])
        self.optim_G.load_state_dict(ck["optim_G"])
        self.optim_D.load_state_dict(ck["optim_D"])
        self.decay_G.load_state_dict(ck["decay_G"])
        self.decay_D.load_state_dict(ck["decay_D"])

    def init_weight(self, g1_weights=None, g2_weights=None, d1_weights=None, d2_weights=None):
        for name, path in (("G1", g1_weights), ("G2", g2_weights), ("D1", d1_weights), ("D2", d2_weights)):
            net = getattr(self, name)
            if path:
                state_dict = torch.load(path, map_location="cpu", weights_only=True)
                net.load_state_dict(state_dict)
                self.logger.info(f"Loaded {name} weights: {path}")
            else:
                net.apply(networks.weights_init)


def _write_png(path, img):
    """cv.imwrite(path, img) for a uint8 HxW or HxWx3 (BGR) array, through PIL (cv2 is not a
    dependency): the PNG holds the same pixel values cv.imwrite would store."""
    from PIL import Image
    os.makedirs(os.path.dirname(path), exist_ok=True)
    arr = np.ascontiguousarray(img[:, :, ::-1]) if img.ndim == 3 else img
    Image.fromarray(arr).save(path)
