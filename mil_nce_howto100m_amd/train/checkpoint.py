"""Checkpoint save / rotate / resume in the reference's exact format.

File ``<root>/<checkpoint_dir>/epoch%04d.pth.tar`` holding
``{"epoch", "state_dict" (keys prefixed 'module.'), "optimizer", "scheduler"}``
(``main_distributed.py:192-200, 289-302``); the newest 10 are kept. Differences, all
format-preserving fixes:

* writes go to a temp file + ``os.replace`` (atomic: a crash never leaves a torn file);
* resume uses ``map_location`` so each rank loads to its own device, not cuda:0;
* ``torch.load(weights_only=True)`` — checkpoints contain only tensors and plain containers;
* callers put barriers around save/resume (rank 0 writes; others wait before reading).
"""
from __future__ import annotations

import glob
import os
from typing import Dict, Optional

import torch


def ckpt_name(epoch: int) -> str:
    return "epoch{:0>4d}.pth.tar".format(epoch)


def add_module_prefix(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    return {(k if k.startswith("module.") else "module." + k): v for k, v in sd.items()}


def strip_module_prefix(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    return {(k[len("module."):] if k.startswith("module.") else k): v for k, v in sd.items()}


def model_state_dict(model: torch.nn.Module) -> Dict[str, torch.Tensor]:
    """Reference-format state dict: fp32 NCDHW weights on CPU, 'module.' prefix (DDP-wrapped)."""
    return add_module_prefix({k: v.detach().cpu().clone() for k, v in model.state_dict().items()})


def save_checkpoint(state: dict, checkpoint_dir: str, epoch: int, n_ckpt: int = 10) -> str:
    os.makedirs(checkpoint_dir, exist_ok=True)
    path = os.path.join(checkpoint_dir, ckpt_name(epoch))
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)
    if epoch - n_ckpt >= 0:
        oldest = os.path.join(checkpoint_dir, ckpt_name(epoch - n_ckpt))
        if os.path.isfile(oldest):
            os.remove(oldest)
    return path


def get_last_checkpoint(checkpoint_dir: str) -> str:
    all_ckpt = glob.glob(os.path.join(checkpoint_dir, "epoch*.pth.tar"))
    return sorted(all_ckpt)[-1] if all_ckpt else ""


def load_checkpoint(path: str, map_location="cpu") -> dict:
    return torch.load(path, map_location=map_location, weights_only=True)


def load_model_weights(model: torch.nn.Module, sd: Dict[str, torch.Tensor], strict: bool = True):
    """Load a training checkpoint's ``state_dict`` or a plain S3D dict (with/without 'module.').

    Writes into the existing parameter storage (``copy_``), so flat optimizer buffers that the
    parameters view into stay valid.
    """
    sd = strip_module_prefix(sd)
    own = model.state_dict()
    missing = [k for k in own if k not in sd]
    unexpected = [k for k in sd if k not in own]
    if strict and (missing or unexpected):
        raise KeyError(f"state_dict mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
    with torch.no_grad():
        for k, v in sd.items():
            if k in own:
                own[k].copy_(v.to(own[k].dtype))
    return missing, unexpected
