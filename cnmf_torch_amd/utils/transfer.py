"""Large device -> host copies through pinned staging buffers.

``tensor.cpu()`` of a multi-GB tensor goes through the runtime's pageable path: one
thread faults in the fresh host pages and copies through small internal bounce buffers
(~3 GB/s measured for the 4 GB corrected expression matrix of the 500k-cell Harmony
stage, profiles/r4d_harmony_*).  :func:`to_host` instead DMA-copies fixed-size chunks
into two pinned buffers on a side stream (chunk i + 1 in flight while chunk i is
unpacked) and unpacks each chunk into the destination with a few threads (numpy's copy
drops the GIL, so the page faults and memcpy of the destination run in parallel).
Bitwise a plain copy; small tensors take ``.cpu()``."""
from __future__ import annotations

import concurrent.futures as cf
import os

import numpy as np
import torch

_MIN_BYTES = 64 << 20
_POOL = None


def _pool():
    global _POOL
    if _POOL is None:
        n = max(1, min(8, (os.cpu_count() or 4) // 2))
        _POOL = cf.ThreadPoolExecutor(max_workers=n, thread_name_prefix="cnmf-d2h")
    return _POOL


def to_host(t: torch.Tensor, chunk_bytes: int = 128 << 20) -> np.ndarray:
    """``t.cpu().numpy()`` for a (large) device tensor, through pinned staging buffers."""
    if not t.is_cuda or t.numel() * t.element_size() < _MIN_BYTES:
        return t.detach().cpu().numpy()
    t = t.detach().contiguous()
    flat = t.view(-1)
    n = flat.numel()
    out = np.empty(tuple(t.shape), dtype=torch.empty(0, dtype=t.dtype).numpy().dtype)
    dst = out.reshape(-1)
    step = max(1, chunk_bytes // t.element_size())
    bufs = [torch.empty(min(step, n), dtype=t.dtype, pin_memory=True) for _ in range(2)]
    evs = [torch.cuda.Event() for _ in range(2)]
    cs = torch.cuda.Stream(t.device)
    cs.wait_stream(torch.cuda.current_stream(t.device))
    pool = _pool()
    nw = pool._max_workers

    def issue(i):
        a = i * step
        b = min(n, a + step)
        with torch.cuda.stream(cs):
            bufs[i % 2][:b - a].copy_(flat[a:b], non_blocking=True)
            evs[i % 2].record(cs)
        return a, b

    nchunk = -(-n // step)
    try:
        cur = issue(0)
        for i in range(nchunk):
            evs[i % 2].synchronize()
            nxt = issue(i + 1) if i + 1 < nchunk else None
            a, b = cur
            src = bufs[i % 2][:b - a].numpy()
            part = -(-(b - a) // nw)
            futs = [pool.submit(np.copyto, dst[a + j:min(b, a + j + part)],
                                src[j:min(b - a, j + part)])
                    for j in range(0, b - a, part)]
            for f in futs:
                f.result()
            cur = nxt
    finally:
        cs.synchronize()     # no copy may still target a staging buffer
    t.record_stream(cs)
    return out
