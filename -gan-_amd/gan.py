"""Drop-in vanilla GAN trainer (reference: train/gan.py ``Train``; config 1 of BASELINE.json).

Step semantics kept (gan.py:26-53, optimizers of train/trainunits.py:18-19):
  * generator step: targets 0.95 + 0.05 U[0,1) drawn first, then z; loss BCE(D(G(z)), targets);
    Adam lr 1e-4, betas (0.5, 0.99);
  * critic step: real targets 0.95 + 0.05 U, fake targets 0.05 U, then z (that draw order);
    G forward under no_grad; BCE real loss and BCE fake loss with separate backward calls
    (their gradients accumulate); Adam lr 4e-4, betas (0.0, 0.99).
BCE is ``torch.nn.BCELoss()`` (mean, logs clamped at -100): ops.bce_loss, csrc/act.hip.

Differences that do not change what is trained (as in wgangp.py): Adam is the fused flat-buffer
kernel; the input gradient the reference leaves in ``gen_imgs.grad`` is not computed; the
critic's weight gradient in the generator step (thrown away at the next critic zero_grad) is not
computed; randomness comes from a pluggable source (rng.py).
"""
from __future__ import annotations

import torch

from . import ops, wgangp
from .optim import FusedAdamW


class Train(wgangp.Train):
    def make_optimizers(self):
        """trainunits.py:18-19: torch.optim.Adam (weight_decay 0)."""
        return (FusedAdamW(self.generator, lr=0.0001, betas=(0.5, 0.99), weight_decay=0.0),
                FusedAdamW(self.discriminator, lr=0.0004, betas=(0.0, 0.99), weight_decay=0.0))

    def generator_backward(self, b_size):
        """gan.py:26-33 without the optimizer step."""
        valid_ = 0.95 + 0.05 * self.rng.rand((b_size, 1))
        self.optimizer_G.zero_grad()
        z = self.rng.randn((b_size, self.nz, 1, 1))
        gen_imgs = self._generate(z)
        with wgangp._frozen(self.discriminator):
            g_loss = ops.bce_loss(self.discriminator(gen_imgs), valid_)
            g_loss.backward()
        return gen_imgs, g_loss

    def discriminator_trainstep(self, images, b_size):
        """gan.py:37-53."""
        real_loss, fake_loss = self.discriminator_backward(images, b_size)
        self.optimizer_D.step()
        return real_loss, fake_loss

    def discriminator_backward(self, images, b_size):
        valid_ = 0.95 + 0.05 * self.rng.rand((b_size, 1))
        fake_ = 0.0 + 0.05 * self.rng.rand((b_size, 1))
        z = self.rng.randn((b_size, self.nz, 1, 1))
        self.optimizer_D.zero_grad()
        with torch.no_grad():
            gen_imgs = self._generate(z)
        real_loss = ops.bce_loss(self.discriminator(images.detach()), valid_)
        real_loss.backward()
        fake_loss = ops.bce_loss(self.discriminator(gen_imgs), fake_)
        fake_loss.backward()
        return real_loss, fake_loss

    def train(self, checkpoints=True):
        """Epoch loop of gan.py:55-77 (display side work left out)."""
        if checkpoints:
            self.load_generator_ckpt("")
            self.load_discriminator_ckpt("")
        for _epoch in range(self.num_epochs):
            for images, _ in self.dataloader:
                images = images.to(self.device)
                b = images.shape[0]
                self.discriminator_trainstep(images, b)
                self.generator_trainstep(b)
