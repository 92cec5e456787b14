"""MI355X-native WGAN-GP hot path for the G13_5 / D9_4 pair (drop-in for the reference's
``generators/generator_13_5.py``, ``discriminators/discriminator_9_4.py`` and
``train/wgangp.py``).  Importing the package loads libganamd.so and fails loudly if it is absent.
"""
from . import _lib  # noqa: F401  (loads libganamd.so or raises)
from .discriminator_9_4 import Discriminator
from .generator_13_5 import Generator
from .optim import FusedAdamW
from .rng import DeviceRNG, ReplayRNG
from .wgangp import Train
from . import wganlazygpR2
from . import generator_3_progan, discriminator_3_wgangp_progan

__all__ = ["Generator", "Discriminator", "Train", "FusedAdamW", "DeviceRNG", "ReplayRNG", "wganlazygpR2", "generator_3_progan", "discriminator_3_wgangp_progan"]
