"""Device selection. One process drives one GPU (``LOCAL_RANK`` picks it);
``LZK_DEVICE`` overrides (``cpu`` / ``cuda`` / ``cuda:N``)."""
from __future__ import annotations

import os

import torch


def default_device() -> torch.device:
    env = os.environ.get("LZK_DEVICE")
    if env:
        return torch.device(env)
    if torch.cuda.is_available():
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    return torch.device("cpu")


def sync(dev=None) -> None:
    d = torch.device(dev) if dev is not None else default_device()
    if d.type == "cuda":
        torch.cuda.synchronize(d)
