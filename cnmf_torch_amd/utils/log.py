"""Package logger.  The reference's user-facing ``print`` messages are
kept verbatim where scripts may parse them ("[Worker i]. Starting task j.", "Combining
factorizations for k=K."); everything else goes through ``logging`` under the
``cnmf_torch_amd`` logger, level from ``CNMF_LOG_LEVEL`` (default WARNING)."""
from __future__ import annotations

import logging
import os

_CONFIGURED = False


def get_logger(name: str = "cnmf_torch_amd") -> logging.Logger:
    global _CONFIGURED
    root = logging.getLogger("cnmf_torch_amd")
    if not _CONFIGURED:
        level = os.environ.get("CNMF_LOG_LEVEL", "WARNING").upper()
        root.setLevel(getattr(logging, level, logging.WARNING))
        if not root.handlers:
            h = logging.StreamHandler()
            rank = os.environ.get("RANK")
            tag = f"[rank {rank}] " if rank is not None else ""
            h.setFormatter(logging.Formatter(f"%(asctime)s {tag}%(name)s %(levelname)s: %(message)s"))
            root.addHandler(h)
        root.propagate = False
        _CONFIGURED = True
    return logging.getLogger(name) if name.startswith("cnmf_torch_amd") else root.getChild(name)
