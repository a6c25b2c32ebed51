"""stcgan_amd -- MI355X-native (gfx950) ST-CGAN hot path.

Drop-in for the reference's STCGAN/networks.py, STCGAN/loss.py and the STCGAN
trainer; every FLOP runs in hand-written HIP kernels of libstcgan_hip.so
(C-ABI: include/stcgan_hip.h).
"""
from . import networks, loss  # noqa: F401
from .networks import get_generator, get_discriminator, weights_init  # noqa: F401

__all__ = ["networks", "loss", "get_generator", "get_discriminator", "weights_init"]
