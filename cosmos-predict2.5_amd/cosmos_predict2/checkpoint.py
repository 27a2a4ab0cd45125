"""Checkpoint loading for the reference's released files (safe loaders only).

DiT: a single .pt state dict with `net.`-prefixed keys (EMA already folded in; the reference loads it
with strict=False and skips `_extra_state`: cosmos_predict2/_src/predict2/utils/model_loader.py:100-177,
text2world_model_rectified_flow.py:761-803). VAE: Wan2.1 `tokenizer.pth` (encoder.*, conv1.*, conv2.*,
decoder.*; wan2pt1.py:648-670). Only `torch.load(weights_only=True)` / safetensors are used.
"""
from __future__ import annotations

from typing import Dict

import torch


def _load(path: str) -> Dict[str, torch.Tensor]:
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file

        return load_file(path)
    obj = torch.load(path, map_location="cpu", weights_only=True)
    for key in ("model", "state_dict"):
        if isinstance(obj, dict) and key in obj and isinstance(obj[key], dict):
            obj = obj[key]
    return obj


def load_dit_checkpoint(path: str) -> Dict[str, torch.Tensor]:
    sd = _load(path)
    return {k: v for k, v in sd.items() if isinstance(v, torch.Tensor) and not k.endswith("_extra_state")}


def load_vae_checkpoint(path: str) -> Dict[str, torch.Tensor]:
    return {k: v for k, v in _load(path).items() if isinstance(v, torch.Tensor)}
