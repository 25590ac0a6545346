"""AnnData on-disk (h5ad) layout over the native HDF5 layer (``_h5io``).

Implements the encoding the reference relies on through scanpy (cnmf.py:519, 545, 698;
preprocess.py:242-243): root ``encoding-type=anndata``; ``X`` as a dense dataset or a
``csr_matrix``/``csc_matrix`` group (``data``/``indices``/``indptr`` + ``shape`` attr);
``obs``/``var`` as ``dataframe`` groups (``_index`` string array, ``column-order``,
numeric/bool/string/categorical columns); ``obsm``/``varm``/``layers``/``uns`` dicts.
Files written here are readable by anndata>=0.8 and vice versa.  ``read_X_rows`` reads a
row range of X (dense hyperslab, or CSR ``indptr`` slice) for streaming large inputs.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import scipy.sparse as sp

from .anndata_lite import AnnData

_NATIVE_ERR = None
try:
    from . import _h5io  # type: ignore
except ImportError as e:  # pragma: no cover - exercised only without a build
    _h5io = None
    _NATIVE_ERR = e


def _lib():
    if _h5io is None:
        raise ImportError(
            "cnmf_torch_amd native h5ad layer is not built (run `python -m cnmf_torch_amd._build`)"
            f": {_NATIVE_ERR}")
    return _h5io


# ----------------------------------------------------------------------------- write
def _set_enc(f, path, etype, ever):
    f.set_attr(path, "encoding-type", etype)
    f.set_attr(path, "encoding-version", ever)


def _write_matrix(f, path: str, X, compression: int) -> None:
    if sp.issparse(X):
        fmt = "csc" if sp.isspmatrix_csc(X) or getattr(X, "format", "") == "csc" else "csr"
        X = X.tocsc() if fmt == "csc" else X.tocsr()
        f.create_group(path)
        _set_enc(f, path, f"{fmt}_matrix", "0.1.0")
        f.set_attr(path, "shape", np.asarray(X.shape, dtype=np.int64))
        f.write_array(path + "/data", np.ascontiguousarray(X.data), compression)
        f.write_array(path + "/indices", np.ascontiguousarray(X.indices), compression)
        f.write_array(path + "/indptr", np.ascontiguousarray(X.indptr), compression)
    else:
        X = np.ascontiguousarray(np.asarray(X))
        f.write_array(path, X, compression)
        _set_enc(f, path, "array", "0.2.0")


def _write_strings(f, path, values) -> None:
    f.write_strings(path, [str(v) for v in values])
    _set_enc(f, path, "string-array", "0.2.0")


def _write_column(f, path: str, col: pd.Series, compression: int) -> None:
    if isinstance(col.dtype, pd.CategoricalDtype):
        f.create_group(path)
        _set_enc(f, path, "categorical", "0.2.0")
        f.set_attr(path, "ordered", bool(col.cat.ordered))
        codes = col.cat.codes.values
        f.write_array(path + "/codes", np.ascontiguousarray(codes), compression)
        _set_enc(f, path + "/codes", "array", "0.2.0")
        cats = col.cat.categories
        if cats.dtype.kind in "iuf":
            f.write_array(path + "/categories", np.asarray(cats.values), compression)
            _set_enc(f, path + "/categories", "array", "0.2.0")
        else:
            _write_strings(f, path + "/categories", cats.values)
        return
    vals = col.values
    if vals.dtype.kind in "iufb":
        f.write_array(path, np.ascontiguousarray(vals), compression)
        _set_enc(f, path, "array", "0.2.0")
    else:
        _write_strings(f, path, vals)


def _write_frame(f, path: str, df: pd.DataFrame, compression: int) -> None:
    f.create_group(path)
    _set_enc(f, path, "dataframe", "0.2.0")
    idx_name = "_index"
    cols = [str(c) for c in df.columns]
    if idx_name in cols:
        idx_name = "__index_level_0__"
    f.set_attr(path, "_index", idx_name)
    f.set_attr(path, "column-order", cols)
    _write_strings(f, f"{path}/{idx_name}", df.index.values)
    for c, name in zip(df.columns, cols):
        _write_column(f, f"{path}/{name}", df[c], compression)


def _write_dict(f, path: str, d: dict, compression: int) -> None:
    f.create_group(path)
    _set_enc(f, path, "dict", "0.1.0")
    for k, v in d.items():
        p = f"{path}/{k}"
        if isinstance(v, dict):
            _write_dict(f, p, v, compression)
        elif isinstance(v, pd.DataFrame):
            _write_frame(f, p, v, compression)
        elif isinstance(v, str):
            f.write_strings(p, [v])
            _set_enc(f, p, "string-array", "0.2.0")
        elif sp.issparse(v) or isinstance(v, np.ndarray):
            _write_matrix(f, p, v, compression)
        elif isinstance(v, (list, tuple)):
            arr = np.asarray(v)
            if arr.dtype.kind in "iufb":
                _write_matrix(f, p, arr, compression)
            else:
                _write_strings(f, p, arr)
        elif isinstance(v, (int, float, bool, np.generic)):
            f.write_array(p, np.asarray(v))
            _set_enc(f, p, "numeric-scalar", "0.2.0")
        # other objects (figures, models) are not serialisable -> skipped, like anndata warns


def write_h5ad(path: str, adata, compression=None) -> None:
    """Write an AnnData(-like) object to ``path`` atomically."""
    from .io import atomic_path

    lib = _lib()
    comp = 4 if compression == "gzip" else int(compression or 0)
    with atomic_path(path, suffix=".h5ad") as tmp:
        f = lib.File(tmp, "w")
        try:
            _set_enc(f, "/", "anndata", "0.1.0")
            _write_matrix(f, "/X", adata.X, comp)
            _write_frame(f, "/obs", adata.obs, comp)
            _write_frame(f, "/var", adata.var, comp)
            for key in ("obsm", "varm", "layers", "obsp", "varp"):
                d = getattr(adata, key, None) or {}
                f.create_group("/" + key)
                _set_enc(f, "/" + key, "dict", "0.1.0")
                for k, v in d.items():
                    if isinstance(v, pd.DataFrame):
                        _write_frame(f, f"/{key}/{k}", v, comp)
                    else:
                        _write_matrix(f, f"/{key}/{k}", v, comp)
            _write_dict(f, "/uns", dict(getattr(adata, "uns", {}) or {}), comp)
        finally:
            f.close()


def write_h5ad_row_blocks(path: str, n_rows: int, var: pd.DataFrame, blocks, sparse: bool,
                          dtype, nnz: int = 0, index_dtype=np.int32, obs=None, obsm=None,
                          uns=None) -> None:
    """Write an h5ad whose X arrives as row blocks, in row order, without ever holding
    the whole matrix: ``blocks`` yields (obs_block DataFrame, X_block) with X_block a
    CSR (``sparse``) or dense array of ``dtype``; ``nnz`` is the total non-zero count of
    a CSR X.  X's datasets are created at their final size and filled by hyperslab
    writes (the native layer's create_dataset / write_rows); obs is written at the end
    (``obs``: the whole frame, the blocks' obs parts are then ignored, may be None).
    ``obsm`` / ``uns``: written as :func:`write_h5ad` does.  Same encoding."""
    from .io import atomic_path

    lib = _lib()
    G = len(var)
    with atomic_path(path, suffix=".h5ad") as tmp:
        f = lib.File(tmp, "w")
        try:
            _set_enc(f, "/", "anndata", "0.1.0")
            if sparse:
                f.create_group("/X")
                _set_enc(f, "/X", "csr_matrix", "0.1.0")
                f.set_attr("/X", "shape", np.asarray([n_rows, G], dtype=np.int64))
                f.create_dataset("/X/data", np.dtype(dtype), [int(nnz)])
                f.create_dataset("/X/indices", np.dtype(index_dtype), [int(nnz)])
                f.create_dataset("/X/indptr", np.dtype(np.int64), [int(n_rows) + 1])
            else:
                f.create_dataset("/X", np.dtype(dtype), [int(n_rows), G])
                _set_enc(f, "/X", "array", "0.2.0")
            obs_parts = []
            r0 = e0 = 0
            for obs_b, Xb in blocks:
                n = Xb.shape[0]
                if sparse:
                    Xb = sp.csr_matrix(Xb)
                    f.write_rows("/X/data", e0, np.ascontiguousarray(Xb.data, dtype=dtype))
                    f.write_rows("/X/indices", e0,
                                 np.ascontiguousarray(Xb.indices, dtype=index_dtype))
                    ip = Xb.indptr.astype(np.int64) + e0
                    f.write_rows("/X/indptr", r0, ip[:-1] if r0 + n < n_rows else ip)
                    e0 += Xb.nnz
                else:
                    f.write_rows("/X", r0, np.ascontiguousarray(np.asarray(Xb), dtype=dtype))
                r0 += n
                if obs is None:
                    obs_parts.append(obs_b)
                del Xb, obs_b      # released before the next block is fetched
            if r0 != n_rows or (sparse and e0 != nnz):
                raise ValueError(f"row blocks gave {r0} rows / {e0} non-zeros, expected "
                                 f"{n_rows} / {nnz}")
            if obs is None:
                obs = pd.concat(obs_parts) if obs_parts else pd.DataFrame()
            _write_frame(f, "/obs", obs, 0)
            _write_frame(f, "/var", var, 0)
            for key in ("obsm", "varm", "layers", "obsp", "varp"):
                f.create_group("/" + key)
                _set_enc(f, "/" + key, "dict", "0.1.0")
                if key == "obsm":
                    for k, v in dict(obsm or {}).items():
                        if isinstance(v, pd.DataFrame):
                            _write_frame(f, f"/obsm/{k}", v, 0)
                        else:
                            _write_matrix(f, f"/obsm/{k}", v, 0)
            _write_dict(f, "/uns", dict(uns or {}), 0)
        finally:
            f.close()


# ----------------------------------------------------------------------------- read
def _enc(attrs: dict) -> str:
    e = attrs.get("encoding-type")
    if e is None and "h5sparse_format" in attrs:  # anndata < 0.7
        return attrs["h5sparse_format"] + "_matrix"
    return e or ""


def _read_matrix(f, path: str):
    if f.kind(path) == "dataset":
        return np.asarray(f.read(path))
    attrs = f.attrs(path)
    enc = _enc(attrs)
    if enc in ("csr_matrix", "csc_matrix"):
        shape = tuple(int(s) for s in np.asarray(attrs.get("shape", attrs.get("h5sparse_shape"))))
        data = f.read(path + "/data")
        indices = f.read(path + "/indices")
        indptr = f.read(path + "/indptr")
        cls = sp.csr_matrix if enc == "csr_matrix" else sp.csc_matrix
        return cls((data, indices, indptr), shape=shape)
    raise ValueError(f"unsupported matrix encoding {enc!r} at {path}")


def _read_column(f, path: str):
    if f.kind(path) == "group":
        attrs = f.attrs(path)
        if _enc(attrs) == "categorical":
            codes = np.asarray(f.read(path + "/codes"))
            cats = f.read(path + "/categories")
            cats = np.asarray(cats) if not isinstance(cats, list) else cats
            return pd.Categorical.from_codes(codes, categories=cats,
                                             ordered=bool(attrs.get("ordered", False)))
        if _enc(attrs) in ("nullable-integer", "nullable-boolean"):
            vals = np.asarray(f.read(path + "/values"))
            mask = np.asarray(f.read(path + "/mask"))
            s = pd.array(vals, dtype="Int64" if _enc(attrs) == "nullable-integer" else "boolean")
            s[mask] = pd.NA
            return s
        raise ValueError(f"unsupported column encoding at {path}")
    v = f.read(path)
    return np.asarray(v, dtype=object) if isinstance(v, list) else np.asarray(v)


def _read_frame(f, path: str) -> pd.DataFrame:
    if f.kind(path) != "group":
        raise ValueError(
            f"{path} is stored in the legacy (anndata<0.7) compound format, which is not "
            "supported; re-save the file with a current anndata")
    attrs = f.attrs(path)
    idx_name = attrs.get("_index", "_index")
    order = attrs.get("column-order", [])
    if isinstance(order, np.ndarray):
        order = list(order)
    index = f.read(f"{path}/{idx_name}") if f.exists(f"{path}/{idx_name}") else None
    cols = {}
    for c in order:
        cols[c] = _read_column(f, f"{path}/{c}")
    n = len(index) if index is not None else (len(next(iter(cols.values()))) if cols else 0)
    idx = pd.Index([str(i) for i in index]) if index is not None else pd.RangeIndex(n).astype(str)
    df = pd.DataFrame(cols, index=idx)
    if order:
        df = df[list(order)]
    return df


def _read_dict(f, path: str) -> dict:
    out = {}
    if not f.exists(path):
        return out
    for k in f.list(path):
        p = f"{path}/{k}"
        try:
            if f.kind(p) == "group":
                enc = _enc(f.attrs(p))
                if enc in ("csr_matrix", "csc_matrix"):
                    out[k] = _read_matrix(f, p)
                elif enc == "dataframe":
                    out[k] = _read_frame(f, p)
                else:
                    out[k] = _read_dict(f, p)
            else:
                v = f.read(p)
                if isinstance(v, list) and len(v) == 1 and _enc(f.attrs(p)) == "string-array":
                    v = v[0]
                out[k] = v
        except (ValueError, OSError):
            continue
    return out


def read_h5ad(path: str, backed=None) -> AnnData:
    """Read an .h5ad file into an :class:`AnnData`."""
    lib = _lib()
    with lib.File(str(path), "r") as f:
        X = _read_matrix(f, "/X") if f.exists("/X") else None
        obs = _read_frame(f, "/obs")
        var = _read_frame(f, "/var")
        obsm = {k: _read_matrix(f, f"/obsm/{k}") for k in f.list("/obsm")} if f.exists(
            "/obsm") else {}
        varm = {k: _read_matrix(f, f"/varm/{k}") for k in f.list("/varm")} if f.exists(
            "/varm") else {}
        layers = {k: _read_matrix(f, f"/layers/{k}") for k in f.list("/layers")} if f.exists(
            "/layers") else {}
        uns = _read_dict(f, "/uns")
    return AnnData(X=X, obs=obs, var=var, obsm=obsm, varm=varm, layers=layers, uns=uns)


def h5ad_shape(path: str) -> tuple[int, int]:
    lib = _lib()
    with lib.File(str(path), "r") as f:
        if f.kind("/X") == "dataset":
            s = f.shape("/X")
            return int(s[0]), int(s[1])
        shp = np.asarray(f.attrs("/X")["shape"])
        return int(shp[0]), int(shp[1])


def read_X_rows(path: str, start: int, stop: int):
    """Rows [start, stop) of X as dense ndarray or CSR, without loading the whole file."""
    lib = _lib()
    with lib.File(str(path), "r") as f:
        if f.kind("/X") == "dataset":
            return np.asarray(f.read("/X", start, stop))
        attrs = f.attrs("/X")
        if _enc(attrs) != "csr_matrix":
            return _read_matrix(f, "/X")[start:stop]
        shape = tuple(int(s) for s in np.asarray(attrs["shape"]))
        stop = min(stop, shape[0])
        indptr = np.asarray(f.read("/X/indptr", start, stop + 1))
        lo, hi = int(indptr[0]), int(indptr[-1])
        data = np.asarray(f.read("/X/data", lo, hi))
        indices = np.asarray(f.read("/X/indices", lo, hi))
        return sp.csr_matrix((data, indices, indptr - lo), shape=(stop - start, shape[1]))


def read_X_row_segments(path: str, segments):
    """Rows of X for a list of [start, stop) segments, concatenated in order (dense
    ndarray or CSR); the file is opened once."""
    lib = _lib()
    parts = []
    with lib.File(str(path), "r") as f:
        dense = f.kind("/X") == "dataset"
        attrs = None if dense else f.attrs("/X")
        if not dense and _enc(attrs) != "csr_matrix":
            full = _read_matrix(f, "/X")
            return np.concatenate([np.asarray(full[a:b]) for a, b in segments]) if segments \
                else np.asarray(full[:0])
        shape = None if dense else tuple(int(x) for x in np.asarray(attrs["shape"]))
        for a, b in segments:
            if dense:
                parts.append(np.asarray(f.read("/X", a, max(a, b))))
                continue
            b = min(max(a, b), shape[0])
            indptr = np.asarray(f.read("/X/indptr", a, b + 1))
            lo, hi = int(indptr[0]), int(indptr[-1])
            data = np.asarray(f.read("/X/data", lo, hi))
            indices = np.asarray(f.read("/X/indices", lo, hi))
            parts.append(sp.csr_matrix((data, indices, indptr - lo), shape=(b - a, shape[1])))
    if dense:
        return np.concatenate(parts) if parts else np.zeros((0, 0))
    return sp.vstack(parts, format="csr")


def read_h5ad_annotations(path: str) -> AnnData:
    """obs/var only (X left as None): what a cell-sharded rank needs besides its rows."""
    lib = _lib()
    with lib.File(str(path), "r") as f:
        obs = _read_frame(f, "/obs")
        var = _read_frame(f, "/var")
    return AnnData(X=None, obs=obs, var=var)
