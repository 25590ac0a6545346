"""Device-resident mirrors of files this process wrote (SURVEY.md §2.2 on-disk contract).

The pipeline's stages hand data to each other through files (prepare writes the
variance-normalised counts, factorize and consensus read them back -- cnmf.py:583,
cnmf.py:860, cnmf.py:1027).  When one process runs several stages, the matrix a stage
just wrote from a device tensor is still exactly that tensor: re-reading 4-8 GB from
disk, casting it on the host and uploading it again is pure overhead (the 500k-cell
Harmony pipeline spent ~2.5 s of its stages on it, profiles/r4d_harmony_*).

``remember(path, tag, value)`` records ``value`` for ``path`` under the file's identity
(inode, size, mtime in ns) right after the write; ``recall(path, tag)`` returns it only
while the file is still that file -- any rewrite, copy over or touch of the path
invalidates the entry, so a reader never sees anything but the file's contents.  The
files are still written and remain the interface between processes (workers, resumed
runs); the mirror only short-cuts readers in the writing process.

Entries are bounded by ``CNMF_RESIDENT_BYTES`` (default: a quarter of the device's
memory; 0 disables), oldest evicted first."""
from __future__ import annotations

import os
import threading
from collections import OrderedDict

_LOCK = threading.Lock()
_CACHE: "OrderedDict[tuple, tuple]" = OrderedDict()   # (realpath, tag) -> (sig, value, nbytes)


def _sig(path: str):
    try:
        st = os.stat(path)
    except OSError:
        return None
    return (st.st_dev, st.st_ino, st.st_size, st.st_mtime_ns)


def _budget() -> int:
    env = os.environ.get("CNMF_RESIDENT_BYTES")
    if env is not None and env != "":
        return int(float(env))
    if not _GPU_TOTAL:
        tot = 0
        try:
            import torch

            if torch.cuda.is_available():
                # hipMemGetInfo (get_device_properties' first call initialises amdsmi,
                # ~0.1 s); asked once per process
                tot = int(torch.cuda.mem_get_info(torch.cuda.current_device())[1])
        except Exception:
            pass
        _GPU_TOTAL.append(tot)
    return _GPU_TOTAL[0] // 4


_GPU_TOTAL: list = []


def _nbytes(value) -> int:
    """Bytes held by a mirror: tensors / arrays, dicts of them, sparse matrices (data +
    indices + indptr), CSR objects with those fields (ops.sparse.DeviceCSR), and
    AnnData-like containers by their X plus the device CSR consensus attaches to them
    (api._device_csr_cached) -- which appears AFTER remember(), so totals are recounted
    on every remember (see there)."""
    if value is None:
        return 0
    if isinstance(value, dict):
        return sum(_nbytes(v) for v in value.values())
    if hasattr(value, "element_size") and hasattr(value, "numel"):
        return int(value.element_size() * value.numel())
    if all(hasattr(value, a) for a in ("data", "indices", "indptr")):
        return sum(_nbytes(getattr(value, a)) for a in ("data", "indices", "indptr"))
    if hasattr(value, "nbytes"):
        return int(value.nbytes)
    if hasattr(value, "X") and hasattr(value, "obs"):
        return _nbytes(value.X) + _nbytes(value.__dict__.get("_cnmf_device_csr"))
    return 0


def wanted(X) -> bool:
    """Whether a dense float32 mirror of the (cells x genes) ``X`` fits the budget."""
    try:
        return int(X.shape[0]) * int(X.shape[1]) * 4 <= _budget()
    except Exception:
        return False


def remember(path: str, tag: str, value) -> bool:
    """Mirror ``value`` as the contents of ``path`` (call right after writing it)."""
    budget = _budget()
    nb = _nbytes(value)
    sig = _sig(path)
    if sig is None or budget <= 0 or nb > budget:
        forget(path)
        return False
    key = (os.path.realpath(path), tag)
    with _LOCK:
        _CACHE.pop(key, None)
        # drop every other tag of this path too (they mirror an older write)
        for k in [k for k in _CACHE if k[0] == key[0]]:
            del _CACHE[k]
        # recounted: an entry may have grown since it was remembered (the device CSR
        # consensus attaches to a remembered TPM AnnData)
        sizes = {k: _nbytes(e[1]) for k, e in _CACHE.items()}
        total = sum(sizes.values())
        while _CACHE and total + nb > budget:
            k, _ = _CACHE.popitem(last=False)
            total -= sizes[k]
        _CACHE[key] = (sig, value, nb)
    return True


def recall(path: str, tag: str):
    """The value remembered for ``path`` if the file is unchanged since, else None."""
    key = (os.path.realpath(path), tag)
    with _LOCK:
        e = _CACHE.get(key)
        if e is None:
            return None
        if _sig(path) != e[0]:
            del _CACHE[key]
            return None
        _CACHE.move_to_end(key)
        return e[1]


def forget(path: str | None = None) -> None:
    """Drop the entries of ``path`` (all entries when None)."""
    with _LOCK:
        if path is None:
            _CACHE.clear()
            return
        rp = os.path.realpath(path)
        for k in [k for k in _CACHE if k[0] == rp]:
            del _CACHE[k]
