"""Checkpoint save / resume of the trainers (reference: train/trainunits.py:58-130).

Kept from the reference: the file naming (``checkpoint/<G name> <D name> <method> epoch_<E>
i_<I>_ckpt.pth``), the fields ``generator_name``, ``discriminator_name``, ``method``, ``epoch``,
``i`` with the same epoch/i carry arithmetic, and ``load_*_ckpt(name)`` reading
``checkpoint/<name>.pth`` and doing nothing when it is absent.

Changed: the reference pickles whole modules and, on load, rebinds
``self.generator`` while the optimizers keep the old parameters (they silently stop training
the loaded network).  Here ``generator`` / ``discriminator`` are ``state_dict()``s keyed by the
reference's own parameter/buffer names (drop-in and reference modules load each other's), they
are loaded IN PLACE (the flat-buffer views and the optimizers stay bound), and the optimizer
moments and step counters are saved too, and so are the device RNG's stream offsets
(``DeviceRNG.state()``: z / noise, eps and synthetic-data streams) and its Philox key (``seed``;
restored on load even when the resuming process was seeded differently), so a resumed run
continues the random sequence instead of redrawing the first run's numbers.  Everything is tensors/str/int, so
``torch.load(..., weights_only=True)`` reads it.

Data parallel: the replicas' parameters and optimizer state are identical, but every rank draws
from its OWN Philox key (bench.py seeds rank r with 4321 + r), so rank 0 writes the file with every
rank's key and offsets (``rng_ranks``, gathered) and each rank resumes its own; a resume at another
world size keeps each rank's own key and takes rank 0's offsets (distinct keys, distinct streams).

Graph-safe: the load writes every tensor in place (parameters, optimizer moments and step counter,
BatchNorm statistics, RNG key and offsets), then refreshes the persistent packed conv-weight copies
(``FlatParams.packs``) that captured graphs launch with -- a graph captured before the load replays
the loaded state (tests/test_resume_gpu.py).
"""
from __future__ import annotations

import os
import pickle

import torch


def _is_dist():
    return torch.distributed.is_available() and torch.distributed.is_initialized()


def _cpu_state(module):
    return {k: v.detach().to("cpu", copy=True) for k, v in module.state_dict().items()}


def _refresh_packed(opt):
    """Parameters were rewritten in place: refresh the persistent GEMM-order weight copies of the
    optimizer's flat buffer, which graphs captured before the load launch with (the eager path
    would repack on the version change; a graph replay does not look)."""
    flat = getattr(opt, "flat", None)
    if flat is not None and hasattr(flat, "packs"):
        flat.epoch += 1
        flat.packs.repack()


def ckpt_path(root, g_name, d_name, method, epoch, i):
    return os.path.join(root, f"{g_name} {d_name} {method} epoch_{epoch} i_{i}_ckpt.pth")


class CheckpointMixin:
    """Mixed into the trainers; needs generator(_name), discriminator(_name), optimizer_G/D,
    and the epoch bookkeeping ``epoch``, ``i``, ``epoch_len``."""

    ckpt_root = "checkpoint"

    def _ckpt_counters(self, epoch, i):
        e = epoch + self.epoch + (i + self.i) // self.epoch_len
        return e, (i + self.i) % self.epoch_len

    def save_ckpt(self, train_name, epoch, i):
        """trainunits.py:58-77 (state_dicts + optimizer state instead of pickled modules)."""
        e, ii = self._ckpt_counters(epoch, i)
        state = {"generator": _cpu_state(self.generator), "generator_name": self.generator_name,
                 "discriminator": _cpu_state(self.discriminator), "discriminator_name": self.discriminator_name,
                 "method": train_name, "epoch": e, "i": ii,
                 "optimizer_G": self.optimizer_G.state_dict(), "optimizer_D": self.optimizer_D.state_dict()}
        rng = getattr(self, "rng", None)
        if hasattr(rng, "state"):
            mine = {"rng": {str(k): v.detach().to("cpu") for k, v in rng.state().items()},
                    "rng_seed": int(rng.seed)}     # the offsets index THIS key's sequence
            state.update(mine)
            if _is_dist():                          # every rank's own key and offsets
                ranks = [None] * torch.distributed.get_world_size()
                torch.distributed.all_gather_object(ranks, mine)
                state["rng_ranks"] = ranks
        path = ckpt_path(self.ckpt_root, self.generator_name, self.discriminator_name, train_name, e, ii)
        err = None
        if not _is_dist() or torch.distributed.get_rank() == 0:
            # data parallel: the replicas are identical, rank 0 writes the file
            try:
                os.makedirs(self.ckpt_root, exist_ok=True)
                torch.save(state, path)
            except Exception as ex:          # noqa: BLE001 -- every rank learns of it below
                err = ex
        if _is_dist():
            # no rank returns before the file is complete, and every rank sees rank 0's failure
            flag = [None if err is None else f"{type(err).__name__}: {err}"]
            torch.distributed.broadcast_object_list(flag, src=0)
            if flag[0] is not None and err is None:
                raise RuntimeError(f"checkpoint save failed on rank 0: {flag[0]}")
        if err is not None:
            raise err
        return path

    def _load(self, name):
        path = os.path.join(self.ckpt_root, name + ".pth")
        if not os.path.isfile(path):
            return None
        try:
            return torch.load(path, map_location="cpu", weights_only=True)
        except pickle.UnpicklingError as e:
            raise RuntimeError(
                f"{path}: not a state_dict checkpoint.  The reference's train/trainunits.py:58-76 pickles whole "
                "nn.Module objects, which are never unpickled here (weights_only=True).  Convert it once where the "
                "reference is importable: ck['generator'] = ck['generator'].state_dict() (same for "
                "'discriminator') and torch.save(ck, path).") from e

    def load_generator_ckpt(self, name):
        """trainunits.py:93-111: also restores epoch / i; loads in place."""
        ck = self._load(name)
        if ck is None:
            return False
        self.generator.load_state_dict(ck["generator"])
        if "optimizer_G" in ck:
            self.optimizer_G.load_state_dict(ck["optimizer_G"])
        _refresh_packed(self.optimizer_G)
        self.epoch, self.i = int(ck["epoch"]), int(ck["i"])
        rng = getattr(self, "rng", None)
        if "rng" in ck and hasattr(rng, "set_state"):
            saved, rekey = ck, True
            if _is_dist():
                ranks, r = ck.get("rng_ranks"), torch.distributed.get_rank()
                if ranks is not None and len(ranks) == torch.distributed.get_world_size():
                    saved = ranks[r]                 # this rank's own key and offsets
                else:
                    rekey = False                    # another world size: keep this rank's own key
            if rekey and "rng_seed" in saved and hasattr(rng, "set_seed") and int(saved["rng_seed"]) != rng.seed:
                rng.set_seed(int(saved["rng_seed"]))  # a process seeded otherwise resumes the saved key
            rng.set_state({int(k): v for k, v in saved["rng"].items()})
        return True

    def load_discriminator_ckpt(self, name):
        """trainunits.py:113-128."""
        ck = self._load(name)
        if ck is None:
            return False
        self.discriminator.load_state_dict(ck["discriminator"])
        if "optimizer_D" in ck:
            self.optimizer_D.load_state_dict(ck["optimizer_D"])
        _refresh_packed(self.optimizer_D)
        return True
