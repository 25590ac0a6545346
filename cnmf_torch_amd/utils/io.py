"""File-level persistence layer (SURVEY.md §1 L4, §2.2 on-disk contract).

Re-implements the reference's DataFrame npz codec (cnmf.py:32-41), TSV writer
(cnmf.py:35-36) and directory helper (cnmf.py:43-51) with two fixes from SURVEY.md
§5.2: every write is atomic (temp file + ``os.replace``), so a killed worker never
leaves a truncated ``.df.npz`` that the resume ledger would count as complete, and
string/number index arrays are stored as plain numpy dtypes so our own files load
with ``allow_pickle=False``.  Files written by the original cnmf (object arrays) are
still readable: ``load_df_from_npz`` retries with pickle enabled for those.
"""
from __future__ import annotations

import contextlib
import errno
import gzip
import io
import os
import tempfile
import threading
import warnings

import numpy as np
import pandas as pd
import yaml


# --------------------------------------------------------------------------- atomic
@contextlib.contextmanager
def atomic_path(final_path: str, suffix: str = ""):
    """Yield a temp path in the destination directory; rename over ``final_path``
    on success, delete on failure.  ``suffix`` keeps extensions numpy/matplotlib
    key off (e.g. ``.npz``)."""
    d = os.path.dirname(os.path.abspath(final_path)) or "."
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".tmp_" + os.path.basename(final_path) + ".", suffix=suffix,
                               dir=d)
    os.close(fd)
    try:
        yield tmp
        os.replace(tmp, final_path)
    except BaseException:
        with contextlib.suppress(OSError):
            os.remove(tmp)
        raise


def write_text_atomic(path: str, text: str) -> None:
    with atomic_path(path) as tmp:
        with open(tmp, "w") as fh:
            fh.write(text)


# --------------------------------------------------------------------------- npz codec
def _plain_array(values) -> np.ndarray:
    """Convert an index/columns array to a non-object dtype when possible."""
    arr = np.asarray(values)
    if arr.dtype != object:
        return arr
    if len(arr) == 0:
        return arr.astype(str)
    if all(isinstance(v, str) for v in arr):
        return arr.astype(str)
    if all(isinstance(v, (int, np.integer)) and not isinstance(v, (bool, np.bool_)) for v in arr):
        return arr.astype(np.int64)
    if all(isinstance(v, (float, np.floating, int, np.integer)) for v in arr):
        return arr.astype(np.float64)
    return arr


def _plain_values(df: pd.DataFrame) -> np.ndarray:
    vals = df.values
    if vals.dtype != object:
        return vals
    # mixed numeric/bool columns (e.g. the replicate ledger) -> int64 when lossless
    kinds = {np.dtype(t).kind for t in df.dtypes}
    if kinds <= {"i", "u", "b"}:
        return df.astype(np.int64).values
    if kinds <= {"i", "u", "b", "f"}:
        return df.astype(np.float64).values
    return vals


NPZ_COMPRESSLEVEL = 1
# Intermediate files under cnmf_tmp/ that only this pipeline re-reads (per-replicate and
# merged spectra): stored uncompressed by default -- float64 spectra barely deflate and
# zlib dominated combine.  Still a standard .npz that np.load reads.
NPZ_TMP_LEVEL = 0


# members at least this large are deflated in parallel chunks (_deflate_parallel)
_PAR_DEFLATE_MIN = 8 << 20
_PAR_DEFLATE_CHUNK = 4 << 20
_DEFLATE_POOL = None
_DEFLATE_LOCK = threading.Lock()


def _deflate_pool():
    """The chunk-deflate threads (their own pool: a caller may itself run on another
    pool's worker)."""
    global _DEFLATE_POOL
    with _DEFLATE_LOCK:
        if _DEFLATE_POOL is None:
            import concurrent.futures as cf

            n = max(2, min(8, (os.cpu_count() or 4) // 2))
            _DEFLATE_POOL = cf.ThreadPoolExecutor(max_workers=n,
                                                  thread_name_prefix="cnmf-deflate")
    return _DEFLATE_POOL


def _deflate_parallel(payload, level: int):
    """(raw deflate stream, crc32) of ``payload`` compressed in independent chunks on a
    thread pool (zlib drops the GIL): every chunk but the last ends with a full flush
    (byte-aligned, no dictionary carried over), so the concatenation is ONE valid deflate
    stream -- the pigz construction.  A 500k-cell usage table (two 40 MB members) took
    ~0.6 s of the Harmony pipeline's consensus on one thread."""
    import zlib

    mv = memoryview(payload)
    n = len(mv)
    parts = [(a, min(n, a + _PAR_DEFLATE_CHUNK)) for a in range(0, n, _PAR_DEFLATE_CHUNK)]

    def comp(i):
        a, b = parts[i]
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        return c.compress(mv[a:b]) + c.flush(zlib.Z_FINISH if i == len(parts) - 1
                                              else zlib.Z_FULL_FLUSH)

    fut = _deflate_pool().map(comp, range(len(parts)))
    crc = zlib.crc32(mv) & 0xFFFFFFFF      # one pass on this thread meanwhile
    return b"".join(fut), crc


def _zip_deflated(path: str, members) -> None:
    """A PKZIP archive of deflated members given as (name, raw deflate stream, crc32,
    uncompressed size) -- what zipfile writes for ZIP_DEFLATED (np.load reads it)."""
    import struct

    out, central, off = [], [], 0
    for name, comp, crc, usize in members:
        nm = name.encode()
        csize = len(comp)
        if csize >= 0xFFFFFFFF or usize >= 0xFFFFFFFF or off >= 0xFFFFFFFF:
            raise ValueError("member too large for the deflated fast path")
        head = struct.pack("<IHHHHHIIIHH", 0x04034B50, 20, 0, 8, 0, 33, crc, csize, usize,
                           len(nm), 0) + nm
        central.append(struct.pack("<IHHHHHHIIIHHHHHII", 0x02014B50, 20, 20, 0, 8, 0, 33,
                                   crc, csize, usize, len(nm), 0, 0, 0, 0, 0o600 << 16, off)
                       + nm)
        out += [head, comp]
        off += len(head) + csize
    cd = b"".join(central)
    with open(path, "wb") as fh:
        fh.writelines(out)
        fh.write(cd)
        fh.write(_zip_end(len(central), len(cd), off))


def _savez_deflate(path: str, arrays: dict, level: int) -> None:
    """np.savez_compressed with a selectable zlib level (numpy hard-codes the default,
    ~4x slower than level 1 on spectra-sized float arrays).  Same member names
    (``<key>.npy``) and ZIP_DEFLATED format, so np.load / the reference read it.
    ``level`` 0 stores the members uncompressed (ZIP_STORED, as np.savez).  Archives
    with a member of >= 8 MB are deflated in parallel chunks (_deflate_parallel)."""
    import zipfile

    if level > 0:
        payloads = {k: npy_bytes(v) for k, v in arrays.items()}
        total = sum(len(b) for b in payloads.values())
        if (max(len(b) for b in payloads.values()) >= _PAR_DEFLATE_MIN
                and total < 0xFFFFFFF0):
            members = []
            for k, b in payloads.items():
                comp, crc = _deflate_parallel(b, level)
                members.append((k + ".npy", comp, crc, len(b)))
            _zip_deflated(path, members)
            return

    comp = zipfile.ZIP_DEFLATED if level > 0 else zipfile.ZIP_STORED
    with zipfile.ZipFile(path, mode="w", compression=comp,
                         compresslevel=level if level > 0 else None, allowZip64=True) as zf:
        for key, arr in arrays.items():
            with zf.open(key + ".npy", "w", force_zip64=True) as fh:
                np.lib.format.write_array(fh, np.asanyarray(arr), allow_pickle=False)


def npy_bytes(arr) -> bytes:
    """The .npy encoding of ``arr`` (pickle-free)."""
    buf = io.BytesIO()
    np.lib.format.write_array(buf, np.ascontiguousarray(arr), allow_pickle=False)
    return buf.getvalue()


def _zip_entry(name: str, payload: bytes, off: int):
    """(local header + name, central-directory record) of one stored ZIP member."""
    import struct
    import zlib

    nm = name.encode()
    crc = zlib.crc32(payload) & 0xFFFFFFFF
    n = len(payload)
    if n >= 0xFFFFFFFF or off >= 0xFFFFFFFF:
        raise ValueError("member too large for the stored-zip fast path")
    head = struct.pack("<IHHHHHIIIHH", 0x04034B50, 20, 0, 0, 0, 33, crc, n, n, len(nm), 0) + nm
    cent = struct.pack("<IHHHHHHIIIHHHHHII", 0x02014B50, 20, 20, 0, 0, 0, 33, crc, n, n,
                       len(nm), 0, 0, 0, 0, 0o600 << 16, off) + nm
    return head, cent


def _zip_end(n_members: int, cd_size: int, cd_off: int) -> bytes:
    import struct

    return struct.pack("<IHHHHIIH", 0x06054B50, 0, 0, n_members, n_members, cd_size, cd_off, 0)


def _zip_stored(members) -> bytes:
    """A minimal PKZIP archive of uncompressed (stored) members -- exactly what
    ``np.savez`` writes (np.load reads it), assembled with one crc32 per member instead
    of zipfile's per-member Python machinery."""
    out, central, off = [], [], 0
    for name, payload in members:
        head, cent = _zip_entry(name, payload, off)
        central.append(cent)
        out += [head, payload]
        off += len(head) + len(payload)
    cd = b"".join(central)
    return b"".join(out) + cd + _zip_end(len(central), len(cd), off)


class NpzTemplate:
    """Writer for many .npz files that share members (the per-replicate spectra files
    all carry the same gene names): the shared members are encoded, checksummed and
    sha256-hashed ONCE, and every file is then [shared members][own members][central
    directory], written atomically with its sha256 continued from the shared prefix.
    A standard stored ZIP: np.load / load_df_from_npz read it."""

    def __init__(self, shared: dict):
        import hashlib

        self.prefix_parts, self.central, off = [], [], 0
        for k, v in shared.items():
            payload = v if isinstance(v, bytes) else npy_bytes(v)
            head, cent = _zip_entry(k + ".npy", payload, off)
            self.prefix_parts += [head, payload]
            self.central.append(cent)
            off += len(head) + len(payload)
        self.prefix_len = off
        self.sha = hashlib.sha256()
        for part in self.prefix_parts:
            self.sha.update(part)

    def write(self, path: str, own: dict) -> tuple[str, int]:
        parts, central, off = [], list(self.central), self.prefix_len
        for k, v in own.items():
            payload = v if isinstance(v, bytes) else npy_bytes(v)
            head, cent = _zip_entry(k + ".npy", payload, off)
            parts += [head, payload]
            central.append(cent)
            off += len(head) + len(payload)
        cd = b"".join(central)
        parts += [cd, _zip_end(len(central), len(cd), off)]
        h = self.sha.copy()
        for part in parts:
            h.update(part)
        with atomic_path(path, suffix=".npz") as tmp:
            with open(tmp, "wb") as fh:
                fh.writelines(self.prefix_parts)
                fh.writelines(parts)
        return h.hexdigest(), off + len(cd) + 22


try:  # native batch writer (csrc/io/npzio.cpp); the Python NpzTemplate is the fallback
    from . import _npzio  # type: ignore
except Exception:  # pragma: no cover - depends on the build
    _npzio = None


def npy_header(shape, dtype) -> bytes:
    """The .npy header bytes of a C-ordered array of ``shape`` / ``dtype``."""
    import numpy.lib.format as fmt

    buf = io.BytesIO()
    fmt.write_array_header_1_0(buf, {"descr": fmt.dtype_to_descr(np.dtype(dtype)),
                                     "fortran_order": False, "shape": tuple(shape)})
    return buf.getvalue()


def write_spectra_batch(paths, data: np.ndarray, offs, ks, columns) -> list[tuple[str, int]]:
    """Write one ``.df.npz`` per replicate -- data rows ``offs[i] : offs[i] + ks[i]`` of the
    float32 matrix ``data``, index 1..K, the shared gene ``columns`` -- atomically, and
    return their (sha256, size).  Native threads when the extension is built (no GIL),
    else the Python :class:`NpzTemplate`."""
    data = np.ascontiguousarray(data, dtype=np.float32)
    G = data.shape[1]
    kset = sorted(set(int(k) for k in ks))
    if _npzio is not None:
        cols = npy_bytes(np.asarray(columns))
        return [tuple(r) for r in _npzio.write_spectra_batch(
            [str(p) for p in paths], data, [int(o) for o in offs], [int(k) for k in ks], cols,
            {k: npy_bytes(np.arange(1, k + 1)) for k in kset},
            {k: npy_header((k, G), np.float32) for k in kset},
            max(1, min(32, (os.cpu_count() or 1))))]
    tmpl = NpzTemplate({"columns": np.asarray(columns)})
    idx = {k: npy_bytes(np.arange(1, k + 1)) for k in kset}
    return [tmpl.write(str(p), {"index": idx[int(k)], "data": data[o:o + int(k)]})
            for p, o, k in zip(paths, offs, ks)]


def read_spectra_batch(paths) -> tuple[np.ndarray, list, np.ndarray] | None:
    """(data (sum K, G) float32, K per file, gene columns) of the replicate ``.df.npz``
    files -- the stored npz :func:`write_spectra_batch` writes -- parsed on native threads
    (csrc/io/npzio.cpp).  None when the extension is missing or a file needs numpy
    (compressed members, other dtypes, object arrays of the original cnmf, gene names
    that differ byte-wise from the first file's): the caller then reads them with numpy."""
    if _npzio is None or not paths:
        return None
    try:
        data, ks, cols = _npzio.read_spectra_batch([str(p) for p in paths],
                                                    max(1, min(32, os.cpu_count() or 1)))
    except ValueError as e:
        if "unsupported" in str(e):
            return None
        raise
    return data, list(ks), np.load(io.BytesIO(cols), allow_pickle=False)


def npz_bytes(arrays: dict, level: int = 0) -> bytes:
    """The bytes of an .npz holding ``arrays`` (same members as :func:`_savez_deflate`).
    Values may be arrays or already-encoded .npy ``bytes`` (shared members such as the
    gene names are encoded once per factorize, not once per file)."""
    if level <= 0:
        return _zip_stored([(k + ".npy", v if isinstance(v, bytes) else npy_bytes(v))
                            for k, v in arrays.items()])
    buf = io.BytesIO()
    _savez_deflate(buf, {k: (np.load(io.BytesIO(v)) if isinstance(v, bytes) else v)
                         for k, v in arrays.items()}, level)
    return buf.getvalue()


def write_bytes_atomic(path: str, data: bytes) -> None:
    with atomic_path(path, suffix=".npz" if path.endswith(".npz") else "") as tmp:
        with open(tmp, "wb") as fh:
            fh.write(data)


def save_arrays_npz_digest(path: str, arrays: dict, level: int = 0) -> tuple[str, int]:
    """Atomically write an .npz of ``arrays``; returns (sha256 hex, size) of the bytes
    written, hashed in memory (no re-read of the file for the replicate manifest)."""
    import hashlib

    data = npz_bytes(arrays, level)
    write_bytes_atomic(path, data)
    return hashlib.sha256(data).hexdigest(), len(data)


def df_npz_arrays(obj: pd.DataFrame) -> dict:
    """The data / index / columns arrays :func:`save_df_to_npz` stores for ``obj``."""
    return {"data": _plain_values(obj), "index": _plain_array(obj.index.values),
            "columns": _plain_array(obj.columns.values)}


def save_df_to_npz(obj: pd.DataFrame, filename: str, level: int | None = None) -> None:
    """Compressed npz with keys data / index / columns -- the cnmf.py:32-33 contract.
    ``level``: zlib level (default NPZ_COMPRESSLEVEL; 0 = stored, for intermediates)."""
    filename = str(filename)
    with atomic_path(filename, suffix=".npz") as tmp:
        _savez_deflate(tmp, {"data": _plain_values(obj),
                             "index": _plain_array(obj.index.values),
                             "columns": _plain_array(obj.columns.values)},
                       NPZ_COMPRESSLEVEL if level is None else int(level))


def load_df_from_npz(filename: str, allow_pickle_fallback: bool = True) -> pd.DataFrame:
    """Inverse of :func:`save_df_to_npz` (cnmf.py:38-41)."""
    filename = str(filename)
    try:
        with np.load(filename, allow_pickle=False) as f:
            return pd.DataFrame(data=f["data"], index=f["index"], columns=f["columns"])
    except ValueError as e:
        if not allow_pickle_fallback or "allow_pickle" not in str(e):
            raise
        # Files produced by the original cnmf store object arrays.
        with np.load(filename, allow_pickle=True) as f:
            return pd.DataFrame(data=f["data"], index=f["index"], columns=f["columns"])


def _tsv_native_args(obj):
    """(corner, columns, index, data) for the native TSV writer when its output is
    byte-identical to ``obj.to_csv(sep="\t")`` -- a plain all-float32 / all-float64 frame
    whose labels need no CSV quoting -- else None."""
    if _npzio is None or not isinstance(obj, pd.DataFrame) or obj.shape[1] == 0:
        return None
    if isinstance(obj.index, pd.MultiIndex) or isinstance(obj.columns, pd.MultiIndex):
        return None
    if obj.columns.name is not None:
        return None
    dts = set(obj.dtypes)
    if len(dts) != 1 or next(iter(dts)) not in (np.dtype(np.float32), np.dtype(np.float64)):
        return None
    lab_kinds = (str, int, np.integer, np.str_)
    idx, cols = list(obj.index), list(obj.columns)
    if not all(isinstance(v, lab_kinds) and not isinstance(v, bool) for v in idx + cols):
        return None
    idx, cols = [str(v) for v in idx], [str(v) for v in cols]
    corner = "" if obj.index.name is None else str(obj.index.name)
    bad = ("\t", "\n", "\r", '"')
    if any(b in s for s in idx + cols + [corner] for b in bad):
        return None
    return corner, cols, idx, np.ascontiguousarray(obj.to_numpy())


def save_df_to_text(obj: pd.DataFrame, filename: str) -> None:
    """Tab-separated text, as cnmf.py:35-36.  All-float frames go through the native
    writer (csrc/io/npzio.cpp write_tsv: the same bytes as pandas' to_csv, formatted on
    native threads; pandas took ~0.16 s of every consensus on the GPU box)."""
    filename = str(filename)
    args = _tsv_native_args(obj)
    with atomic_path(filename) as tmp:
        if args is not None:
            _npzio.write_tsv(tmp, *args)
        else:
            obj.to_csv(tmp, sep="\t")


def check_dir_exists(path: str) -> None:
    """mkdir -p tolerating EEXIST (cnmf.py:43-51)."""
    try:
        os.makedirs(path)
    except OSError as exception:
        if exception.errno != errno.EEXIST:
            raise


# --------------------------------------------------------------------------- yaml
def dump_yaml(obj: dict, path: str) -> None:
    with atomic_path(path) as tmp:
        with open(tmp, "w") as fh:
            yaml.safe_dump(_yaml_clean(obj), fh)


def load_yaml(path: str) -> dict:
    with open(path) as fh:
        return yaml.safe_load(fh)


def _yaml_clean(o):
    if isinstance(o, dict):
        return {str(k): _yaml_clean(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_yaml_clean(v) for v in o]
    if isinstance(o, np.generic):
        return o.item()
    return o


# --------------------------------------------------------------------------- 10x mtx
def _open_maybe_gz(path: str):
    if os.path.exists(path):
        return open(path, "rb")
    if os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rb")
    raise FileNotFoundError(path)


def read_10x_mtx(path: str, var_names: str = "gene_symbols", make_unique: bool = True):
    """Read a 10x Genomics ``matrix.mtx[.gz]`` directory (cnmf.py:520-522 semantics of
    ``sc.read_10x_mtx``): cells x genes CSR float32, gene symbols as var names."""
    import scipy.io
    import scipy.sparse as sp

    from .anndata_lite import AnnData

    with _open_maybe_gz(os.path.join(path, "matrix.mtx")) as fh:
        m = scipy.io.mmread(fh)
    X = sp.csr_matrix(m.T, dtype=np.float32)
    genes_file = None
    for cand in ("features.tsv", "genes.tsv"):
        if os.path.exists(os.path.join(path, cand)) or os.path.exists(
                os.path.join(path, cand + ".gz")):
            genes_file = cand
            break
    if genes_file is None:
        raise FileNotFoundError(f"no features.tsv/genes.tsv in {path}")
    with _open_maybe_gz(os.path.join(path, genes_file)) as fh:
        genes = pd.read_csv(fh, sep="\t", header=None)
    with _open_maybe_gz(os.path.join(path, "barcodes.tsv")) as fh:
        barcodes = pd.read_csv(fh, sep="\t", header=None)[0].astype(str).values
    ids = genes[0].astype(str).values
    symbols = genes[1].astype(str).values if genes.shape[1] > 1 else ids
    names = symbols if var_names == "gene_symbols" else ids
    var = pd.DataFrame(index=pd.Index(names))
    var["gene_ids"] = ids
    if genes.shape[1] > 2:
        var["feature_types"] = genes[2].astype(str).values
    ad = AnnData(X=X, obs=pd.DataFrame(index=pd.Index(barcodes)), var=var)
    if make_unique:
        ad.var_names_make_unique()
    return ad


def read_counts_table(counts_fn: str, densify: bool):
    """Load ``.npz`` (DataFrame codec) or TSV counts into an AnnData (cnmf.py:524-537)."""
    import scipy.sparse as sp

    from .anndata_lite import AnnData

    if counts_fn.endswith(".npz"):
        df = load_df_from_npz(counts_fn)
    else:
        df = pd.read_csv(counts_fn, sep="\t", index_col=0)
    X = df.values if densify else sp.csr_matrix(df.values)
    return AnnData(X=X, obs=pd.DataFrame(index=df.index.astype(str)),
                   var=pd.DataFrame(index=df.columns.astype(str)))


def read_any(path: str, densify: bool = False):
    """Dispatch on extension the way cNMF.prepare does (cnmf.py:518-541)."""
    from .h5ad import read_h5ad

    if path.endswith(".h5ad"):
        return read_h5ad(path)
    if path.endswith(".mtx") or path.endswith(".mtx.gz"):
        return read_10x_mtx(os.path.dirname(path))
    return read_counts_table(path, densify)


# ----------------------------------------------------------------------------- row shards
def count_table_rows(path: str) -> int:
    """Data rows of a TSV counts table (lines after the header), counted in 16 MB reads."""
    n = 0
    last = b"\n"
    with open(path, "rb") as fh:
        while True:
            buf = fh.read(1 << 24)
            if not buf:
                break
            n += buf.count(b"\n")
            last = buf[-1:]
    if last != b"\n":
        n += 1
    return max(0, n - 1)


def _npy_member(z, name: str):
    """(file object positioned at the array data, shape, fortran_order, dtype) of a .npy
    member of an open zip file."""
    fh = z.open(name)
    version = np.lib.format.read_magic(fh)
    if version == (1, 0):
        shape, fortran, dtype = np.lib.format.read_array_header_1_0(fh)
    else:
        shape, fortran, dtype = np.lib.format.read_array_header_2_0(fh)
    return fh, shape, fortran, dtype


def read_npz_df_rows(path: str, a: int, b: int):
    """Rows [a, b) of a DataFrame-codec ``.df.npz`` (save_df_to_npz) without reading the
    others into memory: the ``data`` member is streamed (stored members are sought past,
    deflated ones decompressed and discarded in 16 MB pieces up to row a).  Returns
    (values, index[a:b], columns, n_rows), or None when the member cannot be streamed
    (object arrays of the original cnmf, Fortran order)."""
    import zipfile

    with zipfile.ZipFile(path) as z:
        names = set(z.namelist())
        if "data.npy" not in names:
            return None
        fh, shape, fortran, dtype = _npy_member(z, "data.npy")
        with fh:
            if dtype.hasobject or fortran or len(shape) != 2:
                return None
            n, G = shape
            a, b = max(0, min(a, n)), max(0, min(b, n))
            row_bytes = G * dtype.itemsize
            skip = a * row_bytes
            while skip > 0:
                got = len(fh.read(min(skip, 1 << 24)))
                if got == 0:
                    raise ValueError(f"{path}: truncated data member")
                skip -= got
            raw = fh.read((b - a) * row_bytes)
            vals = np.frombuffer(raw, dtype=dtype).reshape(b - a, G).copy()
        with np.load(path, allow_pickle=False) as f:
            index, columns = f["index"], f["columns"]
    return vals, index[a:b], columns, n


def read_10x_mtx_rows(path: str, a: int | None, b: int | None, rank_of=None,
                      var_names: str = "gene_symbols", make_unique: bool = True):
    """Cells [a, b) of a 10x ``matrix.mtx[.gz]`` directory (genes x cells on disk): the
    coordinate entries are streamed in 4M-entry pieces and only this block's cells kept,
    so a rank never holds more than its own cells.  ``a``/``b`` None: from ``rank_of``
    (n_cells -> (a, b)).  Returns (AnnData of the block, n_cells)."""
    import scipy.sparse as sp

    from .anndata_lite import AnnData

    with _open_maybe_gz(os.path.join(path, "matrix.mtx")) as fh:
        line = fh.readline()
        while line.startswith(b"%"):
            line = fh.readline()
        n_genes, n_cells, _ = (int(v) for v in line.split())
        if a is None:
            a, b = rank_of(n_cells)
        rows_, cols_, vals_ = [], [], []
        for part in pd.read_csv(fh, sep=r"\s+", header=None, chunksize=1 << 22,
                                dtype={0: np.int64, 1: np.int64, 2: np.float64}, engine="c"):
            g = part[0].to_numpy() - 1
            c = part[1].to_numpy() - 1
            keep = (c >= a) & (c < b)
            if keep.any():
                rows_.append(c[keep] - a)
                cols_.append(g[keep])
                vals_.append(part[2].to_numpy()[keep].astype(np.float32))
    r = np.concatenate(rows_) if rows_ else np.zeros(0, np.int64)
    cc = np.concatenate(cols_) if cols_ else np.zeros(0, np.int64)
    v = np.concatenate(vals_) if vals_ else np.zeros(0, np.float32)
    X = sp.csr_matrix((v, (r, cc)), shape=(b - a, n_genes), dtype=np.float32)
    X.sum_duplicates()
    genes_file = None
    for cand in ("features.tsv", "genes.tsv"):
        if os.path.exists(os.path.join(path, cand)) or os.path.exists(
                os.path.join(path, cand + ".gz")):
            genes_file = cand
            break
    if genes_file is None:
        raise FileNotFoundError(f"no features.tsv/genes.tsv in {path}")
    with _open_maybe_gz(os.path.join(path, genes_file)) as fh:
        genes = pd.read_csv(fh, sep="\t", header=None)
    with _open_maybe_gz(os.path.join(path, "barcodes.tsv")) as fh:
        barcodes = pd.read_csv(fh, sep="\t", header=None)[0].astype(str).values[a:b]
    ids = genes[0].astype(str).values
    symbols = genes[1].astype(str).values if genes.shape[1] > 1 else ids
    names = symbols if var_names == "gene_symbols" else ids
    var = pd.DataFrame(index=pd.Index(names))
    var["gene_ids"] = ids
    if genes.shape[1] > 2:
        var["feature_types"] = genes[2].astype(str).values
    ad = AnnData(X=X, obs=pd.DataFrame(index=pd.Index(barcodes)), var=var)
    if make_unique:
        ad.var_names_make_unique()
    return ad, n_cells


def read_rows_any(path: str, rank_of, densify: bool = False):
    """This rank's block of cells of any prepare input (cnmf.py:518-541 formats), read
    without loading the other ranks' cells: ``rank_of(n_rows) -> (a, b)``.  h5ad: partial
    HDF5 reads; 10x mtx: streamed entries; DataFrame npz: streamed ``data`` member; TSV:
    the block's lines.  Returns (AnnData of rows [a, b), n_rows, (a, b))."""
    import scipy.sparse as sp

    from .anndata_lite import AnnData
    from .h5ad import h5ad_shape, read_X_rows, read_h5ad_annotations

    if path.endswith(".h5ad"):
        n_rows, _ = h5ad_shape(path)
        a, b = rank_of(n_rows)
        ann = read_h5ad_annotations(path)
        return AnnData(X=read_X_rows(path, a, b), obs=ann.obs.iloc[a:b], var=ann.var), n_rows, (a, b)
    if path.endswith(".mtx") or path.endswith(".mtx.gz"):
        holder = {}

        def ro(n):
            holder["ab"] = rank_of(n)
            return holder["ab"]
        ad, n_rows = read_10x_mtx_rows(os.path.dirname(path), None, None, rank_of=ro)
        return ad, n_rows, holder["ab"]
    if path.endswith(".npz"):
        import zipfile

        with zipfile.ZipFile(path) as z:
            fh, shape, _, _ = _npy_member(z, "data.npy")
            fh.close()
        n_rows = int(shape[0])
        a, b = rank_of(n_rows)
        got = read_npz_df_rows(path, a, b)
        if got is None:                      # not streamable: whole file (rare)
            full = read_counts_table(path, densify)
            return AnnData(X=full.X[a:b], obs=full.obs.iloc[a:b], var=full.var), n_rows, (a, b)
        vals, index, columns, _ = got
    else:
        n_rows = count_table_rows(path)
        a, b = rank_of(n_rows)
        df = pd.read_csv(path, sep="\t", index_col=0, skiprows=range(1, a + 1), nrows=b - a)
        vals, index, columns = df.values, df.index, df.columns
    X = vals if densify else sp.csr_matrix(vals)
    return AnnData(X=X, obs=pd.DataFrame(index=pd.Index(index).astype(str)),
                   var=pd.DataFrame(index=pd.Index(columns).astype(str))), n_rows, (a, b)
