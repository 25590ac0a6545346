"""A small AnnData container.

The reference passes ``anndata.AnnData`` objects through its whole API
(cnmf.py:531-537, 624-693; preprocess.py:135-439).  anndata is not a dependency of
this framework, so this module provides the subset the pipeline needs: ``X`` (dense
ndarray or scipy CSR/CSC), ``obs``/``var`` DataFrames, ``obsm``/``varm``/``layers``/
``uns`` dicts, label/mask/position indexing on both axes, and h5ad round-trip through
the native HDF5 layer.  Objects that quack like AnnData (e.g. a real anndata object on
a user's machine) are accepted anywhere an AnnData is expected.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import scipy.sparse as sp


def _as_index(n: int, idx, names: pd.Index):
    """Normalise an axis indexer to a positional int array (or slice)."""
    if isinstance(idx, slice):
        return idx
    if isinstance(idx, (pd.Series, pd.Index)):
        idx = idx.values
    if np.isscalar(idx) or isinstance(idx, str):
        idx = [idx]
    arr = np.asarray(idx)
    if arr.dtype == bool:
        if arr.shape[0] != n:
            raise IndexError(f"boolean index of length {arr.shape[0]} for axis of length {n}")
        return np.flatnonzero(arr)
    if arr.dtype.kind in "iu":
        return arr.astype(np.int64)
    # labels
    pos = names.get_indexer(arr)
    if (pos < 0).any():
        missing = list(arr[pos < 0][:5])
        raise KeyError(f"labels not found: {missing}")
    return pos


def _take(X, rows, cols):
    if isinstance(rows, slice) and isinstance(cols, slice):
        return X[rows, cols]
    if sp.issparse(X):
        X = X[rows, :] if not (isinstance(rows, slice) and rows == slice(None)) else X
        return X[:, cols] if not (isinstance(cols, slice) and cols == slice(None)) else X
    if isinstance(rows, slice):
        return X[rows][:, cols]
    if isinstance(cols, slice):
        return X[rows][:, cols]
    return X[np.ix_(rows, cols)]


class AnnData:
    """Annotated data matrix (cells x features)."""

    def __init__(self, X=None, obs: pd.DataFrame | None = None, var: pd.DataFrame | None = None,
                 obsm: dict | None = None, varm: dict | None = None, layers: dict | None = None,
                 uns: dict | None = None, dtype=None):
        if X is not None and not sp.issparse(X):
            X = np.asarray(X)
            if X.ndim == 1:
                X = X.reshape(1, -1)
        if X is not None and dtype is not None:
            X = X.astype(dtype)
        n_obs = X.shape[0] if X is not None else (len(obs) if obs is not None else 0)
        n_var = X.shape[1] if X is not None else (len(var) if var is not None else 0)
        self.X = X
        self.obs = obs.copy() if obs is not None else pd.DataFrame(
            index=pd.RangeIndex(n_obs).astype(str))
        self.var = var.copy() if var is not None else pd.DataFrame(
            index=pd.RangeIndex(n_var).astype(str))
        if len(self.obs) != n_obs or len(self.var) != n_var:
            raise ValueError(
                f"shape mismatch: X {None if X is None else X.shape}, obs {len(self.obs)}, "
                f"var {len(self.var)}")
        self.obsm = dict(obsm or {})
        self.varm = dict(varm or {})
        self.layers = dict(layers or {})
        self.uns = dict(uns or {})

    # ------------------------------------------------------------------ shape/names
    @property
    def shape(self):
        return (len(self.obs), len(self.var))

    @property
    def n_obs(self) -> int:
        return len(self.obs)

    @property
    def n_vars(self) -> int:
        return len(self.var)

    @property
    def obs_names(self) -> pd.Index:
        return self.obs.index

    @obs_names.setter
    def obs_names(self, names):
        self.obs.index = pd.Index(names)

    @property
    def var_names(self) -> pd.Index:
        return self.var.index

    @var_names.setter
    def var_names(self, names):
        self.var.index = pd.Index(names)

    def var_names_make_unique(self, join: str = "-") -> None:
        self.var.index = _make_unique(self.var.index, join)

    def obs_names_make_unique(self, join: str = "-") -> None:
        self.obs.index = _make_unique(self.obs.index, join)

    def __repr__(self) -> str:
        kind = "sparse" if sp.issparse(self.X) else "dense"
        return f"AnnData object with n_obs x n_vars = {self.n_obs} x {self.n_vars} ({kind})"

    # ------------------------------------------------------------------ indexing
    def __getitem__(self, key) -> "AnnData":
        if not isinstance(key, tuple):
            key = (key, slice(None))
        rk, ck = key
        rows = _as_index(self.n_obs, rk, self.obs.index)
        cols = _as_index(self.n_vars, ck, self.var.index)
        X = _take(self.X, rows, cols) if self.X is not None else None
        obs = self.obs.iloc[rows]
        var = self.var.iloc[cols]
        obsm = {k: (v[rows] if not isinstance(v, pd.DataFrame) else v.iloc[rows])
                for k, v in self.obsm.items()}
        varm = {k: (v[cols] if not isinstance(v, pd.DataFrame) else v.iloc[cols])
                for k, v in self.varm.items()}
        layers = {k: _take(v, rows, cols) for k, v in self.layers.items()}
        out = AnnData(X=X.copy() if X is not None and X is self.X else X, obs=obs, var=var,
                      obsm=obsm, varm=varm, layers=layers, uns=dict(self.uns))
        return out

    def copy(self) -> "AnnData":
        return AnnData(X=None if self.X is None else self.X.copy(), obs=self.obs.copy(),
                       var=self.var.copy(),
                       obsm={k: v.copy() for k, v in self.obsm.items()},
                       varm={k: v.copy() for k, v in self.varm.items()},
                       layers={k: v.copy() for k, v in self.layers.items()},
                       uns=dict(self.uns))

    def to_df(self) -> pd.DataFrame:
        X = self.X.toarray() if sp.issparse(self.X) else self.X
        return pd.DataFrame(X, index=self.obs.index, columns=self.var.index)

    # ------------------------------------------------------------------ io
    def write_h5ad(self, filename: str, compression: int | str | None = None) -> None:
        from .h5ad import write_h5ad

        write_h5ad(str(filename), self, compression=compression)

    write = write_h5ad


def _make_unique(index: pd.Index, join: str = "-") -> pd.Index:
    """anndata's var_names_make_unique: second occurrence of 'A' becomes 'A-1', ..."""
    names = list(map(str, index))
    seen: dict[str, int] = {}
    counts = pd.Series(names).value_counts()
    if (counts <= 1).all():
        return pd.Index(names)
    used = set(names)
    out = []
    for n in names:
        if n in seen:
            k = seen[n]
            cand = f"{n}{join}{k}"
            while cand in used:
                k += 1
                cand = f"{n}{join}{k}"
            seen[n] = k + 1
            used.add(cand)
            out.append(cand)
        else:
            seen[n] = 1
            out.append(n)
    return pd.Index(out)


def is_anndata_like(obj) -> bool:
    return all(hasattr(obj, a) for a in ("X", "obs", "var"))


def to_lite(obj) -> AnnData:
    """Convert any AnnData-like object (e.g. a real anndata.AnnData) to ours."""
    if isinstance(obj, AnnData):
        return obj
    if not is_anndata_like(obj):
        raise TypeError("expected an AnnData-like object with X, obs and var")
    return AnnData(X=obj.X, obs=pd.DataFrame(obj.obs), var=pd.DataFrame(obj.var),
                   obsm=dict(getattr(obj, "obsm", {}) or {}), uns=dict(getattr(obj, "uns", {}) or {}))
