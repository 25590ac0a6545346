"""numpy twin of csrc/kernels/philox.h (Philox4x32-10) for the CPU path.

The uniform stream is bit-identical to the device kernel (cnmf_philox_fill); the
Box-Muller normals match to float32 rounding (libm vs device ocml may differ in the
last ulp of the float64 intermediate).  Used so the CPU oracle and the HIP path start
every replicate from the same init.
"""
from __future__ import annotations

import numpy as np

_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = np.uint32(0x9E3779B9)
_W1 = np.uint32(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)

STREAM_H = 0
STREAM_W = 1
STREAM_REFIT = 2


def philox4x32_10(ctr: np.ndarray, k0: int, k1: int) -> np.ndarray:
    """ctr: (n, 4) uint32 -> (n, 4) uint32."""
    c = ctr.astype(np.uint64)
    key0 = np.uint64(k0 & 0xFFFFFFFF)
    key1 = np.uint64(k1 & 0xFFFFFFFF)
    for r in range(10):
        if r:
            key0 = (key0 + np.uint64(_W0)) & _MASK
            key1 = (key1 + np.uint64(_W1)) & _MASK
        p0 = _M0 * c[:, 0]
        p1 = _M1 * c[:, 2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK
        n = np.empty_like(c)
        n[:, 0] = hi1 ^ c[:, 1] ^ key0
        n[:, 1] = lo1
        n[:, 2] = hi0 ^ c[:, 3] ^ key1
        n[:, 3] = lo0
        c = n
    return c.astype(np.uint32)


def _open01(u: np.ndarray) -> np.ndarray:
    return (u.astype(np.float64) + 0.5) * 2.3283064365386963e-10


def philox_matrix(seed: int, stream: int, rows: int, cols: int, mode: int = 0,
                  row_offset: int = 0) -> np.ndarray:
    """(rows x cols) float32 matrix of |N(0,1)| (mode 0) or U(0,1) (mode 1) values,
    element e = row*cols + col drawn from Philox call e // 4, lane e % 4.  With
    ``row_offset`` the rows [row_offset, row_offset+rows) of the canonical matrix are
    returned (cell-sharded init)."""
    total = rows * cols
    e_begin = row_offset * cols
    first = e_begin // 4
    calls = (e_begin + total + 3) // 4 - first
    idx = np.arange(first, first + calls, dtype=np.uint64)
    ctr = np.zeros((calls, 4), dtype=np.uint32)
    ctr[:, 0] = (idx & _MASK).astype(np.uint32)
    ctr[:, 1] = (idx >> np.uint64(32)).astype(np.uint32)
    ctr[:, 2] = np.uint32(stream)
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    v = philox4x32_10(ctr, seed & 0xFFFFFFFF, seed >> 32)
    if mode == 0:
        u = _open01(v)
        ra = np.sqrt(-2.0 * np.log(u[:, 0]))
        rb = np.sqrt(-2.0 * np.log(u[:, 2]))
        tp = 2.0 * np.pi
        out = np.stack([np.abs(ra * np.cos(tp * u[:, 1])), np.abs(ra * np.sin(tp * u[:, 1])),
                        np.abs(rb * np.cos(tp * u[:, 3])), np.abs(rb * np.sin(tp * u[:, 3]))],
                       axis=1)
    else:
        out = _open01(v)
    off = e_begin - first * 4
    return out.reshape(-1)[off:off + total].astype(np.float32).reshape(rows, cols)
