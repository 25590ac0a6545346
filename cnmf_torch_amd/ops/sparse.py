"""Device-resident CSR matrices and the preprocessing reductions over them.

The reference runs these steps on the host through scanpy / sklearn (normalize_total,
scale(zero_center=False), seurat_v3 HVG statistics, StandardScaler mean/var, the
quantile ceiling; cnmf.py:128-247, 670-681; preprocess.py:21-29, 250-338).  Here the
count matrix is uploaded once as CSR and every step is a pass of a HIP kernel over the
stored entries (csrc/kernels/sparse.hip) with the per-row / per-column factors applied
on the fly -- the normalised, subset, scaled or clipped matrices are never materialised
unless a dense copy is asked for (``densify``).

Every function also runs on CPU tensors with plain torch ops; those paths are the test
oracles of the kernels.  On a CUDA tensor the kernel is required (no silent fallback).
"""
from __future__ import annotations

import math

import numpy as np
import scipy.sparse as sp
import torch

from . import _require_native, _stream_ptr, use_native

try:  # the extension is optional on CPU-only hosts
    from . import _hip  # type: ignore
except Exception:  # pragma: no cover
    _hip = None


class DeviceCSR:
    """A (n x m) CSR matrix on a torch device: indptr int64, indices int32, data float32
    or float64 (integer counts are stored as float32, as normalize_total casts them)."""

    def __init__(self, indptr: torch.Tensor, indices: torch.Tensor, data: torch.Tensor, shape,
                 xf: dict | None = None):
        self.indptr = indptr
        self.indices = indices
        self.data = data
        self.xf = dict(xf or {})     # lazy transform of the stored values (see view())
        n_out = self.xf.pop("n_out", None)
        self.shape = (int(shape[0]), int(shape[1] if n_out is None else n_out))
        self.n_stored_cols = int(shape[1])
        self._rows = None

    def view(self, *, n_out: int | None = None, **xf) -> "DeviceCSR":
        """The same stored matrix seen through a transform (row_scale, col_map, col_div,
        clip, max_value, round_mid; see the module docstring), e.g. the scaled HVG
        subset of a TPM matrix -- consumed by every op below without materialising it."""
        V = DeviceCSR(self.indptr, self.indices, self.data, (self.shape[0], self.n_stored_cols),
                      {**self.xf, **xf})
        V.shape = (self.shape[0], int(n_out) if n_out is not None else self.shape[1])
        V._rows = self._rows
        return V

    @classmethod
    def from_scipy(cls, m, device=None, dtype=None) -> "DeviceCSR":
        m = m if sp.isspmatrix_csr(m) else sp.csr_matrix(m)
        dev = torch.device(device) if device is not None else torch.device("cpu")
        if dtype is None:
            dtype = np.float64 if m.data.dtype == np.float64 else np.float32

        def up(a, dt):
            return torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)

        # kernels rely on distinct columns within a row: a matrix scipy has not checked
        # yet is checked on a worker thread while the arrays upload (scipy's check drops
        # the GIL; it was 0.11 s of the 500k-cell Harmony stage, profiles/r6w_*, and a
        # device-side check after the upload exposed the transfers instead, r6zzb)
        if dev.type == "cuda" and getattr(m, "_has_canonical_format", None) is None:
            import concurrent.futures as cf

            with cf.ThreadPoolExecutor(1, thread_name_prefix="cnmf-csr-check") as ex:
                canon = ex.submit(lambda: bool(m.has_canonical_format))
                A = cls(up(m.indptr, np.int64), up(m.indices, np.int32), up(m.data, dtype),
                        m.shape)
                if canon.result():
                    return A
            del A
        if not m.has_canonical_format:
            m = m.copy()
            m.sum_duplicates()
        return cls(up(m.indptr, np.int64), up(m.indices, np.int32), up(m.data, dtype), m.shape)

    def to_scipy(self, data: torch.Tensor | None = None) -> sp.csr_matrix:
        d = (self.data if data is None else data).cpu().numpy()
        return sp.csr_matrix((d, self.indices.cpu().numpy(), self.indptr.cpu().numpy()),
                             shape=self.shape)

    @property
    def device(self) -> torch.device:
        return self.data.device

    @property
    def nnz(self) -> int:
        return int(self.data.numel())

    def row_ids(self) -> torch.Tensor:
        """Row index of every stored entry (int64, CPU oracle paths)."""
        if self._rows is None:
            counts = self.indptr[1:] - self.indptr[:-1]
            self._rows = torch.repeat_interleave(
                torch.arange(self.shape[0], device=self.device), counts)
        return self._rows


def _sorted_distinct(A: DeviceCSR) -> bool:
    """Whether every row's column indices strictly increase (scipy's canonical format),
    checked where ``A`` lives (a test / debugging check: it synchronises the device)."""
    nnz = A.indices.numel()
    if nnz < 2:
        return True
    start = torch.zeros(nnz, dtype=torch.bool, device=A.indices.device)
    p = A.indptr[1:-1]
    start[p[p < nnz]] = True         # first entry of each row (empty rows repeat a position)
    return bool(((A.indices[1:] > A.indices[:-1]) | start[1:]).all())


def _ptr(t):
    return t.data_ptr() if t is not None else 0


def _f64(t, dev):
    if t is None:
        return None
    t = torch.as_tensor(t, dtype=torch.float64)
    return t.to(dev).contiguous()


def _map(col_map, dev):
    if col_map is None:
        return None
    return torch.as_tensor(col_map, dtype=torch.int32).to(dev).contiguous()


def _merge(A, row_scale, col_map, col_div, clip, max_value, round_mid):
    """Explicit transform arguments override the view's own."""
    x = A.xf
    return (row_scale if row_scale is not None else x.get("row_scale"),
            col_map if col_map is not None else x.get("col_map"),
            col_div if col_div is not None else x.get("col_div"),
            clip if clip is not None else x.get("clip"),
            max_value if max_value is not None else x.get("max_value"),
            bool(round_mid or x.get("round_mid", False)))


def _xform_ref(A: DeviceCSR, row_scale, col_map, col_div, clip, max_value, round_mid):
    """(kept mask, output column, transformed float64 value) of every entry -- the torch
    twin of csr_transform (same operation order and roundings)."""
    v = A.data.to(torch.float64)
    cols = A.indices.long()
    if col_map is not None:
        cols = col_map.long()[cols]
    keep = cols >= 0
    c = cols.clamp(min=0)
    if row_scale is not None:
        v = v * row_scale[A.row_ids()]
        if round_mid:
            v = v.float().double()
    if col_div is not None:
        v = v / col_div[c]
    if clip is not None:
        v = torch.minimum(v, clip[c])
    if max_value is not None and math.isfinite(max_value):
        v = torch.clamp(v, max=max_value)
    return keep, c, v


def row_sums(A: DeviceCSR) -> torch.Tensor:
    """Per-row sum of the stored values (float64)."""
    n = A.shape[0]
    if not use_native(A.data):
        out = torch.zeros(n, dtype=torch.float64)
        return out.index_add_(0, A.row_ids(), A.data.double())
    _require_native()
    out = torch.empty(n, dtype=torch.float64, device=A.device)
    _hip.csr_row_sums(A.indptr.data_ptr(), A.data.data_ptr(), int(A.data.dtype == torch.float64),
                      n, out.data_ptr(), _stream_ptr(A.data))
    return out


def col_stats(A: DeviceCSR, *, row_scale=None, col_map=None, n_out: int | None = None,
              col_div=None, clip=None, max_value: float | None = None, round_mid: bool = False,
              center=None):
    """Per output column: (sum v, sum (v - center)^2 or sum v^2, stored-entry count), all
    float64, of the transformed values v (see module docstring).  Deterministic."""
    dev = A.device
    n_out = int(n_out if n_out is not None else A.shape[1])
    row_scale, col_map, col_div, clip, max_value, round_mid = _merge(
        A, row_scale, col_map, col_div, clip, max_value, round_mid)
    rs, cm, cd, cl, ce = (_f64(row_scale, dev), _map(col_map, dev), _f64(col_div, dev),
                          _f64(clip, dev), _f64(center, dev))
    mv = float("inf") if max_value is None else float(max_value)
    if not use_native(A.data):
        keep, c, v = _xform_ref(A, rs, cm, cd, cl, mv, round_mid)
        c, v = c[keep], v[keep]
        dv = v - ce[c] if ce is not None else v
        s = torch.zeros(n_out, dtype=torch.float64).index_add_(0, c, v)
        q = torch.zeros(n_out, dtype=torch.float64).index_add_(0, c, dv * dv)
        k = torch.zeros(n_out, dtype=torch.float64).index_add_(0, c, torch.ones_like(v))
        return s, q, k
    _require_native()
    n = A.shape[0]
    nb = int(_hip.csr_stats_blocks(n))
    part = torch.empty((3, nb, n_out), dtype=torch.float64, device=dev)
    _hip.csr_col_stats(A.indptr.data_ptr(), A.indices.data_ptr(), A.data.data_ptr(),
                       int(A.data.dtype == torch.float64), n, n_out, _ptr(rs), _ptr(cm),
                       _ptr(cd), _ptr(cl), mv, int(round_mid), _ptr(ce), part[0].data_ptr(),
                       part[1].data_ptr(), part[2].data_ptr(), _stream_ptr(A.data))
    tot = part.sum(dim=1)   # fixed-order reduction over workgroups
    return tot[0], tot[1], tot[2]


def mean_var(A: DeviceCSR, ddof: int = 0, **xf):
    """Column mean and variance (ddof 0 or 1) of the transformed matrix, implicit zeros
    included -- sklearn's two-pass sparse scheme (mean_variance_axis: centred squares of
    the stored values + (n - nnz) mean^2, with the rounding correction), which is what
    scanpy's sparse scale and StandardScaler use.  Returns float64 tensors."""
    n = A.shape[0]
    s, _, _ = col_stats(A, **xf)
    mean = s / n
    _, q, k = col_stats(A, center=mean, **xf)
    corr = s - n * mean                       # sum over all n of (x - mean)
    var = (q + (n - k) * mean * mean - corr * corr / n) / n
    var = torch.clamp(var, min=0.0)
    if ddof and n > 1:
        var = var * (n / (n - ddof))
    return mean, var


def transform(A: DeviceCSR, *, row_scale=None, col_map=None, col_div=None, clip=None,
              max_value: float | None = None, round_mid: bool = False,
              out_dtype=torch.float32) -> torch.Tensor:
    """Transformed value of every stored entry (dropped columns -> -1), same layout as
    A.data."""
    dev = A.device
    row_scale, col_map, col_div, clip, max_value, round_mid = _merge(
        A, row_scale, col_map, col_div, clip, max_value, round_mid)
    rs, cm, cd, cl = _f64(row_scale, dev), _map(col_map, dev), _f64(col_div, dev), _f64(clip, dev)
    mv = float("inf") if max_value is None else float(max_value)
    if not use_native(A.data):
        keep, _, v = _xform_ref(A, rs, cm, cd, cl, mv, round_mid)
        v = v.to(out_dtype)
        v[~keep] = -1
        return v
    _require_native()
    out = torch.empty(A.nnz, dtype=out_dtype, device=dev)
    _hip.csr_transform(A.indptr.data_ptr(), A.indices.data_ptr(), A.data.data_ptr(),
                       int(A.data.dtype == torch.float64), A.shape[0], _ptr(rs), _ptr(cm),
                       _ptr(cd), _ptr(cl), mv, int(round_mid), out.data_ptr(),
                       int(out_dtype == torch.float64), _stream_ptr(A.data))
    return out


def densify(A: DeviceCSR, *, n_out: int | None = None, row_scale=None, col_map=None,
            col_div=None, clip=None, max_value: float | None = None, round_mid: bool = False,
            out_dtype=torch.float32) -> torch.Tensor:
    """Dense (n x n_out) matrix of the transformed entries (zeros elsewhere)."""
    dev = A.device
    n_out = int(n_out if n_out is not None else A.shape[1])
    row_scale, col_map, col_div, clip, max_value, round_mid = _merge(
        A, row_scale, col_map, col_div, clip, max_value, round_mid)
    rs, cm, cd, cl = _f64(row_scale, dev), _map(col_map, dev), _f64(col_div, dev), _f64(clip, dev)
    mv = float("inf") if max_value is None else float(max_value)
    out = torch.zeros((A.shape[0], n_out), dtype=out_dtype, device=dev)
    if not use_native(A.data):
        keep, c, v = _xform_ref(A, rs, cm, cd, cl, mv, round_mid)
        out[A.row_ids()[keep], c[keep]] = v[keep].to(out_dtype)
        return out
    _require_native()
    _hip.csr_densify(A.indptr.data_ptr(), A.indices.data_ptr(), A.data.data_ptr(),
                     int(A.data.dtype == torch.float64), A.shape[0], _ptr(rs), _ptr(cm), _ptr(cd),
                     _ptr(cl), mv, int(round_mid), out.data_ptr(), int(out_dtype == torch.float64),
                     n_out, _stream_ptr(A.data))
    return out


def _xf_args(A: DeviceCSR):
    x = A.xf
    dev = A.device
    rs, cm = _f64(x.get("row_scale"), dev), _map(x.get("col_map"), dev)
    cd, cl = _f64(x.get("col_div"), dev), _f64(x.get("clip"), dev)
    mv = x.get("max_value")
    mv = float("inf") if mv is None else float(mv)
    return rs, cm, cd, cl, mv, bool(x.get("round_mid", False))


def spmm(A: DeviceCSR, B: torch.Tensor) -> torch.Tensor:
    """T(A) @ B for B (A.shape[1] x K) -> (n x K) float32 (the refit numerator x W^T)."""
    K = B.shape[1]
    if B.shape[0] != A.shape[1]:
        raise ValueError(f"spmm: B has {B.shape[0]} rows, A has {A.shape[1]} columns")
    rs, cm, cd, cl, mv, rm = _xf_args(A)
    if not use_native(A.data):
        keep, c, v = _xform_ref(A, rs, cm, cd, cl, mv, rm)
        rows, c, v = A.row_ids()[keep], c[keep], v[keep].float()
        out = torch.zeros((A.shape[0], K), dtype=torch.float32)
        return out.index_add_(0, rows, v[:, None] * B.float()[c])
    _require_native()
    if K > 64:   # the CSR kernel takes <= 64 output columns: column blocks of B
        return torch.cat([spmm(A, B[:, a:a + 64]) for a in range(0, K, 64)], dim=1)
    Bf = B.to(device=A.device, dtype=torch.float32).contiguous()
    out = torch.empty((A.shape[0], K), dtype=torch.float32, device=A.device)
    _hip.csr_spmm(A.indptr.data_ptr(), A.indices.data_ptr(), A.data.data_ptr(),
                  int(A.data.dtype == torch.float64), A.shape[0], _ptr(rs), _ptr(cm), _ptr(cd),
                  _ptr(cl), mv, int(rm), Bf.data_ptr(), K, out.data_ptr(), _stream_ptr(A.data))
    return out


def tspmm(A: DeviceCSR, B: torch.Tensor) -> torch.Tensor:
    """T(A)^T @ B for B (n x K) float32/float64 -> (A.shape[1] x K) float64, deterministic
    (the spectra-refit numerator U^T X and the OLS X^T Y)."""
    K = B.shape[1]
    if B.shape[0] != A.shape[0]:
        raise ValueError(f"tspmm: B has {B.shape[0]} rows, A has {A.shape[0]}")
    n_out = A.shape[1]
    rs, cm, cd, cl, mv, rm = _xf_args(A)
    if not use_native(A.data):
        keep, c, v = _xform_ref(A, rs, cm, cd, cl, mv, rm)
        rows, c, v = A.row_ids()[keep], c[keep], v[keep]
        out = torch.zeros((n_out, K), dtype=torch.float64)
        return out.index_add_(0, c, v[:, None] * B.double()[rows])
    _require_native()
    if K > 64:   # the CSR kernel takes <= 64 output columns: column blocks of B
        return torch.cat([tspmm(A, B[:, a:a + 64]) for a in range(0, K, 64)], dim=1)
    Bd = B.to(A.device)
    if Bd.dtype not in (torch.float32, torch.float64):
        Bd = Bd.double()
    Bd = Bd.contiguous()
    nb = int(_hip.csr_tspmm_blocks(A.shape[0]))
    part = torch.empty((nb, n_out, K), dtype=torch.float64, device=A.device)
    _hip.csr_tspmm(A.indptr.data_ptr(), A.indices.data_ptr(), A.data.data_ptr(),
                   int(A.data.dtype == torch.float64), A.shape[0], n_out, _ptr(rs), _ptr(cm),
                   _ptr(cd), _ptr(cl), mv, int(rm), Bd.data_ptr(),
                   int(Bd.dtype == torch.float64), K, part.data_ptr(), _stream_ptr(A.data))
    return part.sum(dim=0)


def kth_nonneg(x: torch.Tensor, k: int) -> float:
    """The k-th smallest (0-based) of the non-negative entries of the float32 tensor x
    (negative entries are ignored), exactly: a 4-pass radix select over the IEEE bit
    patterns (non-negative floats order like their uint32 images)."""
    x = x.reshape(-1)
    if x.dtype != torch.float32:
        raise TypeError("kth_nonneg: float32 input expected")
    if not use_native(x):
        v = x[x >= 0]
        if not 0 <= k < v.numel():
            raise IndexError("kth_nonneg: k out of range")
        return float(torch.kthvalue(v, k + 1).values)
    _require_native()
    hist = torch.zeros(256, dtype=torch.int64, device=x.device)
    prefix, mask, need = 0, 0, int(k)
    for shift in (24, 16, 8, 0):
        hist.zero_()
        _hip.radix_hist(x.data_ptr(), x.numel(), prefix, mask, shift, hist.data_ptr(),
                        _stream_ptr(x))
        h = hist.cpu().numpy()
        cum = np.cumsum(h)
        if need >= int(cum[-1]):
            raise IndexError("kth_nonneg: k out of range")
        b = int(np.searchsorted(cum, need, side="right"))
        need -= int(cum[b - 1]) if b > 0 else 0
        prefix |= b << shift
        mask |= 0xFF << shift
    return float(np.array([prefix], dtype=np.uint32).view(np.float32)[0])


def quantile_with_zeros(vals: torch.Tensor, n_total: int, q: float) -> float:
    """np.quantile(..., q) (linear interpolation) of a virtual vector holding
    ``n_total - n_stored`` zeros plus the non-negative stored values ``vals`` (float32;
    negative entries are dropped columns and do not count as stored)."""
    n_stored = int((vals >= 0).sum()) if vals.numel() else 0
    n_zero = n_total - n_stored
    pos = q * (n_total - 1)
    lo, hi = int(math.floor(pos)), int(math.ceil(pos))
    stored = None
    if vals.dtype != torch.float32:      # float64 values: torch selection on the device
        stored = vals[vals >= 0]

    def at(i):
        if i < n_zero:
            return 0.0
        if stored is not None:
            return float(torch.kthvalue(stored, i - n_zero + 1).values)
        return kth_nonneg(vals, i - n_zero)

    a = at(lo)
    b = at(hi) if hi != lo else a
    return a + (b - a) * (pos - lo)
