"""Drop-in replacement for STCGAN/networks.py on MI355X.

Same factories (``get_generator``, ``get_discriminator``, ``weights_init``),
same module tree and therefore identical ``state_dict`` keys/shapes, so
reference checkpoints (``G1-latest.pt`` ...) load unchanged.  The torch.nn
layers inside the tree only hold parameters and buffers; ``forward`` of the
network runs the whole network as hand-written HIP kernels
(``engine.gen_forward`` / ``engine.disc_forward``) behind one autograd node.

Differences from the reference that a caller can observe: none in values
(parity-tested); odd spatial sizes follow the pad/crop generator of
src/models/stcgan_g.py:120-132 (the STCGAN/networks.py version raises there);
forward also accepts a list/tuple of NCHW tensors, treated as their channel
concatenation without materialising it (what ``torch.cat(..., 1)`` would give).
"""
import torch
import torch.nn as nn

from . import engine
from . import ops

_DTYPES = {"fp32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16, "bfloat16": torch.bfloat16}


@torch.no_grad()
def weights_init(m):
    """custom weights initialization called on network model (STCGAN/networks.py:9-20)"""
    classname = m.__class__.__name__
    if classname.find('Conv') != -1 or classname.find('BatchNorm') != -1:
        nn.init.normal_(m.weight.data, 0.0, 0.02)
        if m.bias is not None:
            nn.init.constant_(m.bias.data, 0)
    elif classname.find('Linear') != -1:
        nn.init.normal_(m.weight.data, 1.0, 0.02)
        if m.bias is not None:
            nn.init.constant_(m.bias.data, 0)


def get_generator(*args, **kwargs):
    return UnetGenerator(*args, **kwargs)


def get_discriminator(*args, **kwargs):
    return NLayerDiscriminator(*args, **kwargs)


class _HipNet(nn.Module):
    """Common runner: compute dtype, packed-weight cache, one autograd node per call."""

    kind = None

    def __init__(self):
        super().__init__()
        self.compute_dtype = torch.float32
        self._pack_cache = {}
        self._plan = None
        # parallel.BucketExchange averaging this network's gradients over the ranks while its backward runs
        # (set by the trainer when world > 1), or None
        self.grad_exchange = None
        self._exchange_spec = None
        # dict reusing gathered inputs across this network's calls on the same tensors (set by the trainer
        # for one train step), or None
        self.input_cache = None
        # stream that consumes this network's input gradients when it runs on a side stream (set by the
        # trainer), or None
        self.grad_consumer = None
        # a call whose output is not used but whose BatchNorm running statistics must advance (the trainer's
        # G-step real-input discriminator calls with loss type "normal"): the layers after the last
        # BatchNorm are skipped and the output is left unwritten
        self.stats_only = False
        # a list (set by the trainer for one call): the call's BatchNorm layers leave their running statistics
        # alone and append what ops.bn_running_update needs to apply the update later (the trainer orders it after
        # another call's, as the reference's call order has it)
        self.defer_running = None

    def set_compute_dtype(self, dtype):
        """'fp32' (default, parity path) or 'bf16' (bf16 operands, fp32 accumulation/BN/master weights)."""
        self.compute_dtype = _DTYPES[dtype] if isinstance(dtype, str) else dtype
        self._pack_cache.clear()
        ops.invalidate_packs()
        return self

    def _run(self, inp):
        sources = list(inp) if isinstance(inp, (list, tuple)) else [inp]
        for s in sources:
            if not s.is_cuda:
                raise RuntimeError("stcgan_amd networks run on the GPU only (HIP kernels); move the model and "
                                   "inputs to a ROCm device")
        if self._plan is None:
            self._plan = self._make_plan()
        params = self._plan.params
        ctrl = (self._plan, self.kind, self.training, self.compute_dtype, self._pack_cache, len(sources),
                self.input_cache, self.grad_consumer, self.stats_only, self.defer_running)
        return engine.NetFn.apply(ctrl, *sources, *params)

    def _apply(self, fn, *args, **kwargs):
        self._pack_cache.clear()
        ops.invalidate_packs()
        self._plan = None
        # the flat gradient buffer (parallel.flat_grads) lives on the parameters' device: a new one is made
        # on the next backward; an exchange bound to the old buffer is dropped with it
        self._flat_grads = None
        ex = self.grad_exchange
        if ex is not None:  # re-made on the new buffer by the next backward (engine.GradWriter)
            self._exchange_spec = (ex.bucket_elems * 4 / (1 << 20), ex.active, ex.on_complete, ex.expected)
        self.grad_exchange = None
        return super()._apply(fn, *args, **kwargs)


class UnetGenerator(_HipNet):
    """Create a Unet-based generator (STCGAN/networks.py:31-76)"""

    kind = "G"

    def __init__(self, in_channels, out_channels, ngf=64, num_downs=8, norm_layer=nn.BatchNorm2d,
                 use_dropout=False):
        super().__init__()
        if norm_layer is not nn.BatchNorm2d:
            raise NotImplementedError("stcgan_amd: only nn.BatchNorm2d is on the ST-CGAN path")
        if use_dropout:
            raise NotImplementedError("stcgan_amd: use_dropout is not on the ST-CGAN path (STCGAN/stcgan.py:34-37)")
        unet_block = UnetSkipConnectionBlock(ngf * 8, ngf * 8, input_nc=None, submodule=None,
                                             norm_layer=norm_layer, innermost=True)
        for _ in range(num_downs - 5):
            unet_block = UnetSkipConnectionBlock(ngf * 8, ngf * 8, input_nc=None, submodule=unet_block,
                                                 norm_layer=norm_layer, use_dropout=use_dropout)
        unet_block = UnetSkipConnectionBlock(ngf * 4, ngf * 8, input_nc=None, submodule=unet_block,
                                             norm_layer=norm_layer)
        unet_block = UnetSkipConnectionBlock(ngf * 2, ngf * 4, input_nc=None, submodule=unet_block,
                                             norm_layer=norm_layer)
        unet_block = UnetSkipConnectionBlock(ngf, ngf * 2, input_nc=None, submodule=unet_block,
                                             norm_layer=norm_layer)
        self.model = UnetSkipConnectionBlock(out_channels, ngf, input_nc=in_channels, submodule=unet_block,
                                             outermost=True, norm_layer=norm_layer)

    def _make_plan(self):
        return engine.GenPlan(self)

    def forward(self, input):
        """Standard forward: input NCHW fp32 (or a list of NCHW tensors to concatenate)."""
        return self._run(input)


class UnetSkipConnectionBlock(nn.Module):
    """Parameter container with the reference block's layer layout (STCGAN/networks.py:79-143).
    Executed only as part of UnetGenerator (the whole U-Net is one fused HIP schedule)."""

    def __init__(self, outer_nc, inner_nc, input_nc=None, submodule=None, outermost=False, innermost=False,
                 norm_layer=nn.BatchNorm2d, use_dropout=False):
        super().__init__()
        self.outermost = outermost
        self.innermost = innermost
        use_bias = isinstance(norm_layer, nn.InstanceNorm2d)  # always False, as in the reference
        if input_nc is None:
            input_nc = outer_nc
        downconv = nn.Conv2d(input_nc, inner_nc, kernel_size=4, stride=2, padding=1, bias=use_bias)
        downrelu = nn.LeakyReLU(0.2, True)
        downnorm = norm_layer(inner_nc)
        uprelu = nn.ReLU(True)
        upnorm = norm_layer(outer_nc)
        if outermost:
            upconv = nn.ConvTranspose2d(inner_nc * 2, outer_nc, kernel_size=4, stride=2, padding=1)
            model = [downconv, submodule, uprelu, upconv, nn.Tanh()]
        elif innermost:
            upconv = nn.ConvTranspose2d(inner_nc, outer_nc, kernel_size=4, stride=2, padding=1, bias=use_bias)
            model = [downrelu, downconv, uprelu, upconv, upnorm]
        else:
            upconv = nn.ConvTranspose2d(inner_nc * 2, outer_nc, kernel_size=4, stride=2, padding=1, bias=use_bias)
            model = [downrelu, downconv, downnorm, submodule, uprelu, upconv, upnorm]
        self.model = nn.Sequential(*model)

    def forward(self, x):
        raise RuntimeError("stcgan_amd: UnetSkipConnectionBlock runs only inside UnetGenerator.forward")


class NLayerDiscriminator(_HipNet):
    """PatchGAN discriminator (STCGAN/networks.py:147-192)."""

    kind = "D"

    def __init__(self, in_channels, ndf=64, n_layers=3, norm_layer=nn.BatchNorm2d, use_sigmoid=False):
        super().__init__()
        if norm_layer is not nn.BatchNorm2d:
            raise NotImplementedError("stcgan_amd: only nn.BatchNorm2d is on the ST-CGAN path")
        if use_sigmoid:
            raise NotImplementedError("stcgan_amd: use_sigmoid=True is not on the ST-CGAN path "
                                      "(STCGAN/stcgan.py:39,41)")
        use_bias = isinstance(norm_layer, nn.InstanceNorm2d)
        kw, padw = 4, 1
        sequence = [nn.Conv2d(in_channels, ndf, kernel_size=kw, stride=2, padding=padw), nn.LeakyReLU(0.2, True)]
        nf_mult = 1
        for n in range(1, n_layers):
            nf_mult_prev = nf_mult
            nf_mult = min(2 ** n, 8)
            sequence += [nn.Conv2d(ndf * nf_mult_prev, ndf * nf_mult, kernel_size=kw, stride=2, padding=padw,
                                   bias=use_bias),
                         norm_layer(ndf * nf_mult), nn.LeakyReLU(0.2, True)]
        nf_mult_prev = nf_mult
        nf_mult = min(2 ** n_layers, 8)
        sequence += [nn.Conv2d(ndf * nf_mult_prev, ndf * nf_mult, kernel_size=kw, stride=1, padding=padw,
                               bias=use_bias),
                     norm_layer(ndf * nf_mult), nn.LeakyReLU(0.2, True)]
        sequence += [nn.Conv2d(ndf * nf_mult, 1, kernel_size=kw, stride=1, padding=padw)]
        self.model = nn.Sequential(*sequence)

    def _make_plan(self):
        return engine.DiscPlan(self)

    def forward(self, input):
        return self._run(input)
