"""Drop-in lazy-GP + R1/R2 trainer (reference: train/wganlazygpR2.py ``Train``, optimizers of
train/trainunits.py:18-19).

Step semantics kept (wganlazygpR2.py:17-77):
  * generator step: -mean D(G(z)), Adam lr 1e-4, betas (0.5, 0.99), no weight decay;
  * critic step ``idx``: no-grad G forward, real loss -mean D(x), fake loss mean D(G(z)); when
    ``idx % 5 == 0`` additionally R1 = 5 * mean_i |grad_x D(x_i)|^2 on the real batch, R2 the same
    on the fake batch, and GP = 10 * 5 * mean((|grad D(x_hat)| - 1)^2) on eps-interpolated samples
    (eps ~ U[0,1) per sample, drawn after z and the generator noise); Adam lr 4e-4, betas
    (0.0, 0.99).  Returns (real_loss, fake_loss, gp, r2_reg_r, r2_reg_f) with zeros [1] for the
    terms a step does not compute.

Differences that do not change what is trained (same kind as wgangp.py's):
  * The reference runs up to five backward calls per critic step; their gradients accumulate,
    so one backward of the summed objective gives the same parameter gradients.
  * The critic sees the real, fake (and interpolated) batches as ONE pass of 2B (3B) samples with
    per-segment MiniBatchStdDev (Discriminator.forward ``segments``): every other layer is
    per-sample, so the outputs, the per-sample input gradients that R1/R2/GP square, and the
    summed weight gradients are those of the reference's separate passes.
  * The input gradients the reference leaves in ``images.grad`` / ``gen_imgs.grad`` are never
    read (dead work, skipped); as in wgangp.py the critic's weight gradient in the generator step
    is not computed.
"""
from __future__ import annotations

import torch

from . import critic, ops, wgangp
from .discriminator_9_4 import Discriminator
from .optim import FusedAdamW

LAZY_INTERVAL = 5      # wganlazygpR2.py:56,65,71: regularisers every 5th critic step
REG_WEIGHT = 5         # R1 / R2 weight (:58, :67) and the lazy GP multiplier (:72)
GP_LAMBDA = 10         # :72


class Train(wgangp.Train):
    """``precision="bf16"`` (config 4 of BASELINE.json: "bf16 with fp32 GP"): the plain critic
    steps and the generator steps run their conv / linear GEMMs with bf16 operands (fp32
    accumulation, fp32 activations, weights, gradients and optimizer state); the regularised
    critic steps -- R1, R2 and the gradient penalty with their double backward -- stay fp32.
    The reference has no mixed precision: the bf16 path is checked against the
    fp32 fixtures at a documented looser tolerance (tests/test_models_gpu.py)."""

    def __init__(self, *args, precision: str = "fp32", **kw):
        assert precision in ("fp32", "bf16"), precision
        self.precision = precision
        super().__init__(*args, **kw)

    def make_optimizers(self):
        """trainunits.py:18-19: torch.optim.Adam (weight_decay 0)."""
        return (FusedAdamW(self.generator, lr=0.0001, betas=(0.5, 0.99), weight_decay=0.0),
                FusedAdamW(self.discriminator, lr=0.0004, betas=(0.0, 0.99), weight_decay=0.0))

    def discriminator_trainstep(self, images, b_size, idx):
        """wganlazygpR2.py:48-77."""
        out = self.discriminator_backward(images, b_size, idx)
        self.optimizer_D.step()
        return out

    def generator_backward(self, b_size):
        with ops.math_mode(self.precision):
            return super().generator_backward(b_size)

    def discriminator_backward(self, images, b_size, idx):
        self.optimizer_D.zero_grad()
        z = self.rng_g.randn((b_size, self.nz, 1, 1))
        plain = idx % LAZY_INTERVAL != 0
        with ops.math_mode(self.precision if plain else "fp32"), torch.no_grad():
            gen_imgs = self._generate(z)
        images = images.detach()
        if plain:
            with ops.math_mode(self.precision):
                pred = self.discriminator(torch.cat([images, gen_imgs]), segments=2)
                real_loss = -torch.mean(pred[:b_size])
                fake_loss = torch.mean(pred[b_size:])
                (real_loss + fake_loss).backward()
            zero = torch.zeros(1, device=images.device)
            return real_loss, fake_loss, zero, zero.clone(), zero.clone()
        eps = self.rng.rand((b_size,)).view(b_size, 1, 1, 1)
        x_interp = (1 - eps) * images + eps * gen_imgs
        if isinstance(self.discriminator, Discriminator):
            # one pass of each sweep of the critic program (critic.py) over the three segments:
            # loss weights -1/B (real), +1/B (fake), 0 (interpolated) folded into the adjoint seed
            x = torch.cat([images, gen_imgs, x_interp]).detach()
            w = torch.cat([torch.full((b_size,), -1.0 / b_size, device=x.device),
                           torch.full((b_size,), 1.0 / b_size, device=x.device),
                           torch.zeros(b_size, device=x.device)])
            pred, (r2_reg_r, r2_reg_f, gp) = critic.regularised_step(
                self.discriminator, x, 3, w,
                [(0.0, float(REG_WEIGHT), 1), (0.0, float(REG_WEIGHT), 1), (1.0, float(GP_LAMBDA * REG_WEIGHT), 0)])
            real_loss = -torch.mean(pred[:b_size])
            fake_loss = torch.mean(pred[b_size:2 * b_size])
            return real_loss, fake_loss, gp, r2_reg_r, r2_reg_f
        x = torch.cat([images, gen_imgs, x_interp]).detach().requires_grad_()
        pred = self.discriminator(x, segments=3)
        grad = torch.autograd.grad(pred.sum(), x, create_graph=True, retain_graph=True, only_inputs=True)[0]
        real_loss = -torch.mean(pred[:b_size])
        fake_loss = torch.mean(pred[b_size:2 * b_size])
        # R1 = 5 mean |g|^2 (real), R2 = 5 mean |g|^2 (fake), GP = 10 * 5 mean (|g| - 1)^2 (interp):
        # each one fused kernel pair (ops.GradPenalty) on its contiguous batch slice of the gradient
        r2_reg_r = ops.grad_penalty(grad[:b_size], 0.0, float(REG_WEIGHT), 1)
        r2_reg_f = ops.grad_penalty(grad[b_size:2 * b_size], 0.0, float(REG_WEIGHT), 1)
        gp = ops.grad_penalty(grad[2 * b_size:], 1.0, float(GP_LAMBDA * REG_WEIGHT), 0)
        (real_loss + fake_loss + r2_reg_r + r2_reg_f + gp).backward()
        return real_loss, fake_loss, gp, r2_reg_r, r2_reg_f

    def train(self, checkpoints=True):
        """Epoch loop of wganlazygpR2.py:79-121 (resume from ``checkpoint/.pth`` if present; the
        reference saves no checkpoint here, :121 is commented out; display side work left out)."""
        if checkpoints:
            self.load_generator_ckpt("")
            self.load_discriminator_ckpt("")
        for _epoch in range(self.num_epochs):
            for i, (images, _) in enumerate(self.dataloader):
                images = images.to(self.device)
                b = images.shape[0]
                self.discriminator_trainstep(images, b, i)
                self.generator_trainstep(b)
