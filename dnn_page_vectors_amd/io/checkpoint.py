"""Checkpoints in the reference experiment layout, stored as safetensors + JSON.

Reference artefacts (dssm_cnn_v2/cnn_dssm_th.py:193,199-206, config.py:41-75):

    {trained_model_dir}/weights.{epoch:02d}.hdf5      per-epoch ModelCheckpoint (model + optimizer)
    {trained_model_dir}/cnn_model_dssm.h5             final model + optimizer
    {trained_model_dir}/cnn_dssm_model_only.json      architecture
    {trained_model_dir}/cnn_dssm_model_weights.h5     final weights only

Here the same stems with ``.safetensors`` (h5py is unavailable and pickles are not
used), plus ``trainer_state.json`` (epoch, step, optimizer step, data cursor, RNG) so a
run can RESUME — the reference never reloads a checkpoint.  Rank 0 writes; every rank
loads.  Files are written to a temp name and renamed (atomic on POSIX).
"""
from __future__ import annotations

import glob
import json
import os
import re
from typing import Dict, Optional, Tuple

import torch
from safetensors.torch import load_file, save_file

from ..parallel import dist as pdist
from ..utils.fs import create_dir

EPOCH_TPL = "weights.{epoch:02d}.safetensors"
FINAL_FULL = "cnn_model_dssm.safetensors"
FINAL_ARCH = "cnn_dssm_model_only.json"
FINAL_WEIGHTS = "cnn_dssm_model_weights.safetensors"
STATE = "trainer_state.json"


def _atomic_save(tensors: Dict[str, torch.Tensor], path: str, meta: Optional[Dict[str, str]] = None) -> None:
    tmp = path + ".tmp"
    save_file({k: v.detach().contiguous().cpu() for k, v in tensors.items()}, tmp, metadata=meta)
    os.replace(tmp, path)


def _weights(trainer) -> Dict[str, torch.Tensor]:
    return {f"param/{n}": p.detach() for n, p in trainer.model.named_parameters()}


def _full(trainer) -> Dict[str, torch.Tensor]:
    d = _weights(trainer)
    d["optim/m"] = trainer.opt.m
    d["optim/v"] = trainer.opt.v
    return d


def save_epoch(trainer, directory: str, epoch: int, extra_state: Optional[dict] = None) -> str:
    """Per-epoch checkpoint (ModelCheckpoint analogue). Returns the path (rank 0)."""
    path = os.path.join(directory, EPOCH_TPL.format(epoch=epoch))
    if pdist.info().is_main:
        create_dir(directory)
        _atomic_save(_full(trainer), path, {"epoch": str(epoch)})
        st = dict(trainer.state())
        st["checkpoint"] = os.path.basename(path)
        if extra_state:
            st.update(extra_state)
        tmp = os.path.join(directory, STATE + ".tmp")
        with open(tmp, "w") as f:
            json.dump(st, f, indent=2)
        os.replace(tmp, os.path.join(directory, STATE))
    pdist.barrier()
    return path


def save_final(trainer, directory: str) -> Tuple[str, str, str]:
    full = os.path.join(directory, FINAL_FULL)
    arch = os.path.join(directory, FINAL_ARCH)
    wts = os.path.join(directory, FINAL_WEIGHTS)
    if pdist.info().is_main:
        create_dir(directory)
        _atomic_save(_full(trainer), full)
        _atomic_save(_weights(trainer), wts)
        with open(arch, "w") as f:
            json.dump(trainer.model.architecture(), f, indent=2)
    pdist.barrier()
    return full, arch, wts


def load_weights(model: torch.nn.Module, path: str, strict: bool = True) -> None:
    """Load ``param/*`` tensors into the model in place (works with flat-buffer views)."""
    sd = load_file(path)
    params = dict(model.named_parameters())
    missing = [n for n in params if f"param/{n}" not in sd]
    if strict and missing:
        raise KeyError(f"checkpoint {path} lacks {missing}")
    with torch.no_grad():
        for n, p in params.items():
            k = f"param/{n}"
            if k in sd:
                p.copy_(sd[k].to(p.device, p.dtype))
    from ..models.base import bump_generation

    bump_generation()


def load_full(trainer, path: str) -> None:
    load_weights(trainer.model, path)
    sd = load_file(path)
    if "optim/m" in sd:
        trainer.opt.m.copy_(sd["optim/m"].to(trainer.opt.m.device))
        trainer.opt.v.copy_(sd["optim/v"].to(trainer.opt.v.device))


def latest_epoch_checkpoint(directory: str) -> Optional[str]:
    files = glob.glob(os.path.join(directory, "weights.*.safetensors"))
    best, be = None, -1
    for f in files:
        m = re.search(r"weights\.(\d+)\.safetensors$", f)
        if m and int(m.group(1)) > be:
            best, be = f, int(m.group(1))
    return best


def resume(trainer, directory: str) -> bool:
    """Restore the latest per-epoch checkpoint + trainer state. Returns True if resumed."""
    path = latest_epoch_checkpoint(directory)
    stf = os.path.join(directory, STATE)
    if path is None or not os.path.exists(stf):
        return False
    with open(stf) as f:
        st = json.load(f)
    want = os.path.join(directory, st.get("checkpoint", os.path.basename(path)))
    load_full(trainer, want if os.path.exists(want) else path)
    trainer.load_state(st)
    return True


class ModelCheckpoint:
    """Callback: save ``weights.{epoch:02d}.safetensors`` at each epoch end (1-based like Keras' format)."""

    def __init__(self, directory: str, every: int = 1):
        self.directory = directory
        self.every = every

    def on_epoch_end(self, trainer, epoch: int, logs: dict) -> None:
        if (epoch + 1) % self.every == 0:
            save_epoch(trainer, self.directory, epoch + 1, {"logs": logs})
