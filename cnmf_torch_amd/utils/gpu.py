"""Process-wide answer to "is a HIP GPU visible?" -- torch.cuda.is_available() is a HIP
device-count query (~0.5-4 ms per call); the stages ask it many times (91 calls, 0.06 s,
in the 500k-cell preprocess, profiles/r5j_*)."""
from __future__ import annotations

import torch

_VISIBLE: list = []


def visible() -> bool:
    if not _VISIBLE:
        _VISIBLE.append(bool(torch.cuda.is_available()))
    return _VISIBLE[0]
