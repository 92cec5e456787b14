"""Drop-in WGAN-GP trainer (reference: train/wgangp.py ``Train``).

Same step semantics as train/wgangp.py:20-71: zero_grad placement, the generator forward under
``no_grad`` in the critic step, real/fake critic losses with separate ``backward()`` calls, the
gradient penalty on eps-interpolated samples with ``autograd.grad(create_graph=True)`` and
lambda = 10, ``sqrt`` then ``- center``, batch mean, AdamW (G lr 1e-4, D lr 4e-4, betas
(0.5, 0.999)).

Differences that do not change what is trained:
  * AdamW is the fused flat-buffer kernel (optim.py).
  * The critic's input gradient on the fake batch (left in ``gen_imgs.grad`` by
    wgangp.py:65-67 and never read) is not computed.
  * In the generator step the critic's parameters are frozen for the backward: the reference
    computes D's weight gradients there and throws them away at the next critic zero_grad
    ("dead D wgrad"); we do not compute them.
  * Randomness comes from a pluggable source (rng.py) so runs can replay a seeded sequence.
  * The GUI / image-grid / checkpoint side work of train/trainunits.py is not part of the hot
    path; ``train()`` runs the step loop only.
"""
from __future__ import annotations

import contextlib

import torch

from . import critic, ops
from .checkpoint import CheckpointMixin
from .discriminator_9_4 import Discriminator
from .optim import FusedAdamW
from .rng import DeviceRNG


@contextlib.contextmanager
def _frozen(module):
    ps = [p for p in module.parameters() if p.requires_grad]
    for p in ps:
        p.requires_grad_(False)
    try:
        yield
    finally:
        for p in ps:
            p.requires_grad_(True)


class Train(CheckpointMixin):
    def __init__(self, dataloader, device, num_epochs, nz, generator, generator_name, discriminator,
                 discriminator_name, rng=None):
        self.dataloader = dataloader
        self.device = torch.device(device)
        self.num_epochs = num_epochs
        self.nz = nz
        self.generator, self.generator_name = generator, generator_name
        self.discriminator, self.discriminator_name = discriminator, discriminator_name
        self.rng = rng if rng is not None else DeviceRNG(self.device)
        self.optimizer_G, self.optimizer_D = self.make_optimizers()
        # epoch bookkeeping of train/trainunits.py:25-28 (checkpoint names and resume)
        self.epoch, self.i = 0, 0
        try:
            self.epoch_len = max(1, len(dataloader))
        except TypeError:
            self.epoch_len = 1

    def make_optimizers(self):
        """train/wgangp.py:17-18: AdamW (weight_decay 0.01), G lr 1e-4, D lr 4e-4, betas (0.5, 0.999)."""
        return (FusedAdamW(self.generator, lr=0.0001, betas=(0.5, 0.999)),
                FusedAdamW(self.discriminator, lr=0.0004, betas=(0.5, 0.999)))

    @property
    def rng_g(self):
        """The generator's z and in-forward noise source: stream 1 of ``rng`` (DeviceRNG.fork), so
        a fake batch made on a second HIP stream never shares a Philox counter with the critic
        step's eps draws on the first; ReplayRNG forks to itself (the reference's one sequence)."""
        r = self.rng
        c = self.__dict__.get("_rng_g")
        if c is None or c[0] is not r:
            fork = getattr(r, "fork", None)
            c = self.__dict__["_rng_g"] = (r, fork(1) if fork is not None else r)
        return c[1]

    def _generate(self, z):
        hub = getattr(self.generator, "noise_hub", None)      # G13_5's in-forward noise (progan has none)
        if hub is not None:
            hub.attach(self.rng_g)
        return self.generator(z)

    def generator_trainstep(self, b_size):
        """train/wgangp.py:20-27."""
        gen_imgs, g_loss = self.generator_backward(b_size)
        self.optimizer_G.step()
        return gen_imgs, g_loss

    def generator_backward(self, b_size):
        """generator_trainstep up to (not including) the optimizer step."""
        self.optimizer_G.zero_grad()
        z = self.rng_g.randn((b_size, self.nz, 1, 1))
        gen_imgs = self._generate(z)
        with _frozen(self.discriminator):
            g_loss = -torch.mean(self.discriminator(gen_imgs))
            g_loss.backward()
        return gen_imgs, g_loss

    def discriminator_loss(self, real_pred, fake_pred):
        return torch.mean(fake_pred) - torch.mean(real_pred)

    def gradient_penalty(self, x_real, x_fake, batch_size, device=None, center=1.0):
        """train/wgangp.py:34-43."""
        eps = self.rng.rand((batch_size,)).view(batch_size, 1, 1, 1)
        x_interp = ((1 - eps) * x_real + eps * x_fake).detach()
        if not isinstance(self.discriminator, Discriminator):     # e.g. the progan critic
            x_interp.requires_grad_()
            d_out = self.discriminator(x_interp)
            grad = torch.autograd.grad(outputs=d_out.sum(), inputs=x_interp, create_graph=True, retain_graph=True,
                                       only_inputs=True)[0]
            return ops.grad_penalty(grad, center, 1.0, 0)
        # (compute_grad2(d_out, x_interp).sqrt() - center).pow(2).mean() as the critic program of
        # critic.py: forward, input-gradient sweep and the fused penalty now; the returned value's
        # backward() runs the double backward as two explicit sweeps (no autograd graph of D)
        return critic.gradient_penalty(self.discriminator, x_interp, center, 1.0, 0)

    def compute_grad2(self, d_out, x_in):
        """train/wgangp.py:45-54."""
        batch_size = x_in.size(0)
        grad_dout = torch.autograd.grad(outputs=d_out.sum(), inputs=x_in, create_graph=True, retain_graph=True,
                                        only_inputs=True)[0]
        grad_dout2 = grad_dout.pow(2)
        assert grad_dout2.size() == x_in.size()
        return grad_dout2.view(batch_size, -1).sum(1)

    def discriminator_trainstep(self, images, b_size):
        """train/wgangp.py:56-71."""
        out = self.discriminator_backward(images, b_size)
        self.optimizer_D.step()
        return out

    def generate_fake(self, b_size):
        """The critic step's fake batch (wgangp.py:58-59): z draw, then G under no_grad.  It
        depends on the generator's weights only, so a data-parallel driver may compute the NEXT
        critic step's batch on a second stream while this step's gradient all-reduce and
        optimizer update run (bench.py)."""
        z = self.rng_g.randn((b_size, self.nz, 1, 1))
        with torch.no_grad():
            return self._generate(z)

    def generate_fakes(self, n, b_size):
        """The fake batches of n critic steps from ONE generator forward over n * b_size samples
        (wgangp.py:58-59 n times).  G's only cross-sample coupling is train-mode BatchNorm, so the
        forward runs with segmented BatchNorm (ops.bn_segments): each b_size block is normalised by
        its own statistics and the running statistics take the n updates in order -- the
        reference's n separate calls, as one wider launch per layer.  The z and noise values are
        drawn as one block, so they are other samples of the same distributions than n separate
        draws would give (the per-stream Philox order is fixed, so a replay draws the same ones)."""
        z = self.rng_g.randn((n * b_size, self.nz, 1, 1))
        with torch.no_grad(), ops.bn_segments(n):
            return self._generate(z).chunk(n)

    def discriminator_backward(self, images, b_size, gen_imgs=None):
        """discriminator_trainstep up to (not including) the optimizer step.  ``gen_imgs``: a fake
        batch made beforehand by generate_fake (default: made here, in the reference's order)."""
        self.optimizer_D.zero_grad()
        if gen_imgs is None:
            gen_imgs = self.generate_fake(b_size)
        gen_imgs.requires_grad_()
        # The real and fake batches go through the critic as ONE pass of 2B samples (two
        # MiniBatchStdDev segments, see Discriminator.forward): the critic is per-sample apart
        # from that layer, so the outputs and the summed weight gradients are those of the
        # reference's two forward/backward calls (wgangp.py:60-66), with one backward.  The input
        # gradient the reference leaves in gen_imgs.grad is never read (dead work, skipped).
        pred = self.discriminator(torch.cat([images, gen_imgs.detach()]), segments=2)
        pred_r, pred_f = pred[:b_size], pred[b_size:]
        real_loss = -torch.mean(pred_r)
        fake_loss = torch.mean(pred_f)
        (real_loss + fake_loss).backward()
        gp = 10 * self.gradient_penalty(images, gen_imgs, b_size, self.device)
        gp.backward()
        return real_loss, fake_loss, gp

    def train(self, checkpoints=True):
        """Epoch loop of train/wgangp.py:73-95: resume from ``checkpoint/.pth`` if present, one
        critic step + one generator step per batch, a checkpoint after every epoch (display and
        image-grid side work left out)."""
        if checkpoints:
            self.load_generator_ckpt("")
            self.load_discriminator_ckpt("")
        for epoch in range(self.num_epochs):
            for images, _ in self.dataloader:
                images = images.to(self.device)
                b = images.shape[0]
                self.discriminator_trainstep(images, b)
                self.generator_trainstep(b)
            if checkpoints:
                self.save_ckpt("WGANGP", epoch + 1, 0)
