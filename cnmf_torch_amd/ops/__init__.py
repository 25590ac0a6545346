"""Op layer: one entry point per hot operation, dispatched by device.

* CUDA/HIP tensors -> the hand-written gfx950 kernels in ``_hip`` (csrc/kernels).
  If the extension is missing on a GPU run the op raises; there is no silent
  fallback to eager PyTorch for a native op.
* CPU tensors -> the PyTorch reference implementations in :mod:`.reference`, which
  are also the numerics oracle the GPU tests compare against (fp32 and fp64).

Every native op validates shapes/strides/dtypes on the host before launching, so a
kernel is never handed an operand layout it does not assume.
"""
from __future__ import annotations

import contextlib
import os
import threading
from typing import NamedTuple

import numpy as np
import torch

from . import reference

import importlib

_HIP_ERR: Exception | None = None
try:  # the HIP runtime must come from torch's copy -> import torch first (done above)
    _hip = importlib.import_module(__name__ + "._hip")
except Exception as e:  # pragma: no cover - depends on the build
    _hip = None
    _HIP_ERR = e

ALGO_MU = 0
ALGO_HALS = 1
ALGOS = {"mu": ALGO_MU, "hals": ALGO_HALS}


def native_available() -> bool:
    return _hip is not None


def native_error() -> Exception | None:
    return _HIP_ERR


def _require_native():
    if _hip is None:
        raise RuntimeError(
            "cnmf_torch_amd HIP extension is not available on a GPU run "
            f"(build it with `python -m cnmf_torch_amd._build`): {_HIP_ERR}")
    return _hip


# Per-op debug / tuning knobs, read ONCE (at import, or by refresh_env()): every op
# consults them, and os.environ lookups were ~0.5 ms of host time per bench step.
_ENV_KEYS = ("CNMF_FORCE_TORCH_OPS", "CNMF_SOLVE_COOP", "CNMF_GEMM_VARIANT", "CNMF_GEMM_KSPLIT",
             "CNMF_GEMM_STAGES", "CNMF_GEMM_BK", "CNMF_SOLVE_PIPE", "CNMF_KL_FP16")
_ENV: dict = {}


def refresh_env() -> None:
    """Re-read the CNMF_* per-op knobs from the environment."""
    _ENV.clear()
    _ENV.update({k: os.environ.get(k) for k in _ENV_KEYS})


refresh_env()


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` lives on the GPU (the HIP path is then mandatory) -- except inside
    :func:`eager_ops`, the explicit, logged routing of ranks no kernel covers."""
    if t.device.type != "cuda":
        return False
    if _ENV["CNMF_FORCE_TORCH_OPS"] == "1":  # debugging aid only, never default
        return False
    if getattr(_TLS, "eager", False):
        return False
    _require_native()
    return True


@contextlib.contextmanager
def eager_ops():
    """Within this context (per host thread) every op runs its PyTorch reference
    (ops/reference.py) on the operands' own device.  This is the routing for factor ranks
    the native kernels do not cover (K > 128 Frobenius MU, K > 64 HALS / KL, K > 56 IS and
    general beta (models.nmf_base.kernel_max_rank);
    the reference's -k is unbounded, cnmf.py:1417): the caller logs it per job
    (models.nmf.NMFBatchSolver.run, models.refit).  Covered ranks never take it."""
    prev = getattr(_TLS, "eager", False)
    _TLS.eager = True
    try:
        yield
    finally:
        _TLS.eager = prev


def eager_active() -> bool:
    return bool(getattr(_TLS, "eager", False))


# raw current-stream pointer without constructing a torch.cuda.Stream per op (700 per
# bench step through torch.cuda.current_stream)
_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream_ptr(t: torch.Tensor) -> int:
    if _RAW_STREAM is not None and t.device.type == "cuda":
        return _RAW_STREAM(t.get_device())
    return torch.cuda.current_stream(t.device).cuda_stream



def _native_dtype_k(op: str, dtype: torch.dtype, K: int, max_k: int) -> None:
    """A GPU operand outside what the native kernel handles is an error, never a silent
    switch to eager PyTorch (module contract)."""
    if dtype != torch.float32:
        raise TypeError(f"{op}: the native gfx950 kernel computes in float32, got {dtype}")
    if K > max_k:
        raise ValueError(f"{op}: K={K} exceeds the native kernel's maximum {max_k}")


def _check_block_view(name: str, t: torch.Tensor, R: int, K: int, n: int):
    if t.dim() != 3 or tuple(t.shape) != (R, K, n):
        raise ValueError(f"{name}: expected shape {(R, K, n)}, got {tuple(t.shape)}")
    if t.dtype != torch.float32:
        raise TypeError(f"{name}: HIP solve requires float32, got {t.dtype}")
    if n > 1 and t.stride(2) != 1:
        raise ValueError(f"{name}: innermost (column) stride must be 1, got {t.stride()}")


# ----------------------------------------------------------------------------- solve
def solve(algo: str, x: torch.Tensor, numer: torch.Tensor, gram: torch.Tensor,
          rep_index: torch.Tensor | None = None, max_iter: int = 1, tol: float = -1.0,
          l1_num: float = 0.0, l1_den: float = 0.0, l2: float = 0.0, eps: float = 1e-16,
          lin_out: torch.Tensor | None = None, quad_out: torch.Tensor | None = None,
          iters_out: torch.Tensor | None = None, nsplit: int = 1, conv_mode: int = 0,
          check_every: int = 10, variant: str = "auto",
          active: torch.Tensor | None = None, coop: int | str = "auto",
          planes: torch.Tensor | None = None, planes_colmul: torch.Tensor | None = None,
          gram_of: torch.Tensor | None = None, planes_n: int = 3,
          numer_slabs: int = 1, numer_slab_stride: int = 0,
          numer_scale: torch.Tensor | None = None, numer_base: torch.Tensor | None = None,
          numer_out: torch.Tensor | None = None, gram_parts: torch.Tensor | None = None,
          gram_parts_n: int = 0, gram_out: torch.Tensor | None = None,
          gram_parts_out: torch.Tensor | None = None, coop_device_gen: bool = False) -> int:
    """In-place fused inner solve on ``x`` (R, K, n) given ``numer`` (R, K, n) and
    ``gram`` (R, K, K); see csrc/kernels/solve.hip for the update rules.

    ``gram_of`` (R, K, m) instead of ``gram`` (pass None): the system matrix is
    F F^T of this factor -- the matrix-core kernel forms it in its prologue (no separate
    Gram launch), the other kernels get it from :func:`gram`.

    Only replicates listed in ``rep_index`` (int32, default all) are touched.
    ``nsplit > 1`` runs a single fixed step with columns split over blocks (batch mode).
    ``conv_mode`` 0: stop when ||dx||/(||x||+eps) < tol (checked every step);
    1: stop when the block objective's relative change over ``check_every`` steps < tol.
    ``iters_out`` ACCUMULATES the steps taken (zero it for per-call counts).
    ``active`` (int32, one flag per replicate): replicates with 0 are left untouched.
    ``coop``: number S of workgroups cooperating on ONE replicate's columns while still
    converging as a unit (cross-workgroup deterministic reductions, see coop_sum2 in
    solve.hip); "auto" picks S so that all S*nblocks workgroups are co-resident on the
    256 CUs, 1 disables.  Results are independent of S up to fp32 summation order.
    ``variant``: "auto" runs MU with K <= 16 on the matrix-core kernel (solve_mfma.hip:
    Gram x on v_mfma_f32_16x16x4_f32, iterate in VGPRs) whenever its slices fit, else
    the VALU kernels ("stream" / "reg" force those; "mfma" forces the former).
    ``planes`` (>= planes_n, R*K, cols_pad) int16, optional: the kernel's epilogue also writes the
    final x (times ``planes_colmul`` per column) as exact bf16 planes -- the A operand of
    the next split-precision GEMM (ops.gemm_planes) -- zeroing columns [n, cols_pad).
    ``planes_n``: how many of the three planes to write (the GEMM reads only its
    ``gemm_a_planes(Kd)`` A planes; the rest would be dead stores).
    MU with l1 = l2 = 0, the block-objective stop and K <= 16 runs the software-pipelined
    matrix-core kernel (solve_pipe.hip) unless ``CNMF_SOLVE_PIPE=0``.

    Fused operands (pipelined kernel only; a launch that cannot take them raises):
    ``numer_slabs`` / ``numer_slab_stride``: ``numer`` is slab 0 of that many raw split-K
    partials (gemm_planes(raw_slab=...)) ``numer_slab_stride`` floats apart, summed in
    slice order, times ``numer_scale`` (per column), plus ``numer_base`` (R, K, n);
    ``numer_out`` (R, K, n) receives that sum.  ``gram_parts`` (R, >= gram_parts_n, K, K):
    the system matrix is ``gram`` (optional base) + the sum of the first ``gram_parts_n``
    partial Grams; ``gram_out`` (R, K, K) receives it.  ``gram_parts_out`` (R, >= S, K, K):
    slice s of the launch writes its partial Gram sum_cols x x^T of the final x there.
    ``coop_device_gen``: cooperative launches tag their granules from a device-side
    generation the kernel itself advances (pipelined kernel only), so a launch captured
    in a HIP graph needs no zeroing of the granules per replay.
    Returns S, the number of column slices per replicate the launch used.
    """
    a = ALGOS[algo]
    R, K, n = x.shape
    fused = (numer_slabs > 1 or numer_scale is not None or numer_base is not None
             or numer_out is not None or gram_parts is not None or gram_out is not None
             or gram_parts_out is not None or coop_device_gen)
    if fused and not use_native(x):
        raise ValueError("solve: fused operands need the HIP kernels (CUDA tensors)")
    if gram is None and gram_parts is not None:
        pass
    elif gram is None:
        if gram_of is None or gram_of.shape[:2] != (R, K):
            raise ValueError("solve: pass gram (R, K, K) or gram_of (R, K, m)")
    elif gram_of is not None:
        raise ValueError("solve: gram and gram_of are exclusive")
    if gram is None and not use_native(x):
        gram = torch.bmm(gram_of, gram_of.transpose(1, 2))
    if not use_native(x):
        reference.solve(a, x, numer, gram, rep_index, max_iter, tol, l1_num, l1_den, l2,
                        eps, lin_out, quad_out, iters_out, nsplit, conv_mode, check_every,
                        active)
        if planes is not None:
            split_planes(x.reshape(R * K, n), planes[:min(int(planes_n), planes.shape[0])],
                         col_mul=planes_colmul)
        return 1
    h = _hip
    if solve_any_k(a, K):
        # ranks beyond the register-tiled kernels: library Gram-x GEMM + solve_any.hip
        if fused or variant == "mfma":
            raise ValueError(f"solve: K={K} runs the rank-general solve (solve_any.hip), "
                             "which takes no fused operands / variant='mfma'")
        if gram is None:
            gram = _gram_op(gram_of, active=active)
        _solve_any(a, x, numer, gram, rep_index, max_iter, tol, l1_num, l1_den, l2, eps,
                   lin_out, quad_out, iters_out, nsplit, conv_mode, check_every, active)
        if planes is not None:
            split_planes(x.reshape(R * K, n), planes[:min(int(planes_n), planes.shape[0])],
                         col_mul=planes_colmul)
        return 1
    # a GPU operand the kernels do not cover is an error, never a silent eager fallback:
    # fp32 only; K in 1..32 or a padded wide rank (the engine pads K <= 64 to a multiple
    # of 8 and K <= 128 to a multiple of 16, models/nmf.py native_rank)
    _native_dtype_k("solve", x.dtype, K, h.solve_max_k())
    if not h.solve_native_k(K):
        raise ValueError(f"solve: K={K} has no kernel instantiation (pad it with zero "
                         "components, see models.nmf.native_rank)")
    if K > 64 and a != 0:
        raise ValueError(f"solve: K={K} > 64 runs the matrix-core MU solve only "
                         f"(algo={algo!r}); use algo='mu' or 'bpp'")
    _check_block_view("x", x, R, K, n)
    _check_block_view("numer", numer, R, K, n)
    if gram is not None:
        if gram.shape != (R, K, K) or gram.dtype != torch.float32:
            raise ValueError(f"gram: expected float32 {(R, K, K)}, got {gram.dtype} "
                             f"{tuple(gram.shape)}")
        gram = gram.contiguous()
    elif gram_of is not None:
        _check_block_view("gram_of", gram_of, R, K, gram_of.shape[2])
    src = gram if gram is not None else (gram_of if gram_of is not None else gram_parts)
    devs = {x.device, numer.device, src.device}
    if len(devs) != 1:
        raise ValueError(f"solve operands on different devices: {devs}")
    if rep_index is not None:
        if rep_index.dtype != torch.int32 or rep_index.device != x.device:
            raise ValueError("rep_index must be int32 on the same device")
        nblocks = int(rep_index.numel())
        ri = rep_index.data_ptr()
    else:
        nblocks, ri = R, 0
    if nblocks == 0 or n == 0:
        return 0
    if nsplit > 1 and max_iter != 1:
        raise ValueError("nsplit > 1 requires max_iter == 1 (no convergence test)")
    for name, t, dt in (("lin_out", lin_out, torch.float32), ("quad_out", quad_out, torch.float32),
                        ("iters_out", iters_out, torch.int32), ("active", active, torch.int32)):
        if t is not None and (t.dtype != dt or t.numel() < R or not t.is_contiguous()):
            raise ValueError(f"{name}: expected contiguous {dt} with >= {R} elements")
    if nsplit > 1:
        for t in (lin_out, quad_out):
            if t is not None:
                t.zero_()
    f_args = _fused_solve_args(R, K, n, x, numer, numer_slabs, numer_slab_stride, numer_scale,
                               numer_base, numer_out, gram_parts, gram_parts_n, gram_out,
                               gram_parts_out) if fused else (1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)
    # matrix-core variant (csrc/kernels/solve_mfma.hip): MU with K <= 16 whenever every
    # slice fits one 256-thread workgroup's register tiles; four of its workgroups are
    # co-resident per CU, so its cooperative budget is 4x the 1024-thread one
    S = None
    rpl = 0
    pipe_ok = (a == 0 and conv_mode == 1 and nsplit <= 1 and not (l1_num or l1_den or l2)
               and _ENV["CNMF_SOLVE_PIPE"] != "0" and h.solve_pipe_k(K))
    if variant in ("auto", "mfma") and a == 0 and h.solve_mfma_max_cols(K) > 0:
        S = _mfma_split(n, nblocks, K, nsplit, coop, x.device)
    if S is None and pipe_ok and variant in ("auto", "mfma"):
        # the pipelined kernel alone (K > 16, or K <= 16 when every replicate's slices
        # do not fit at once): co-resident rounds of `rpl` replicates
        plan = _pipe_plan(n, nblocks, K, coop, x.device)
        if plan is not None:
            S, rpl = plan
            if gram is None and gram_of is not None:
                gram = _gram_op(gram_of, active=active)
                gram_of = None
    if fused and (S is None or not pipe_ok or gram_of is not None
                  or h.solve_pipe_tiles(K, -(-n // S)) == 0):
        raise ValueError("solve: fused operands need the pipelined MU kernel (K <= 64, "
                         "l1 = l2 = 0, conv_mode 1, cooperative slices that fit)")
    if fused and gram_parts_out is not None and gram_parts_out.shape[1] < S:
        raise ValueError(f"gram_parts_out: {gram_parts_out.shape[1]} slots < {S} slices")
    if S is not None:
        vcode = 5 if _ENV["CNMF_SOLVE_PIPE"] == "0" else 3
    elif gram is None:      # a VALU kernel: form the Gram first
        gram = _gram_op(gram_of, active=active)
    if S is not None:
        pass
    elif variant == "mfma":
        raise ValueError(f"solve: variant 'mfma' does not cover algo={algo} K={K} n={n} "
                         f"with {nblocks} replicates")
    else:
        vcode = {"auto": 0, "stream": 1, "reg": 2}[variant]
        S = 1
        if nsplit <= 1:
            S = _coop_split(n, nblocks, x.device) if coop == "auto" else max(1, int(coop))
        if S > 1 and nblocks * S > _coop_resident(x.device):
            raise ValueError(f"coop={S} x {nblocks} blocks exceeds co-resident workgroups")
    n_slice = (n + S - 1) // S
    threads = min(h.solve_max_threads(K), max(64, ((min(n_slice, 4096 * 4) + 63) // 64) * 64))
    ws_slots = ws_count = ws_flag = 0
    epochs = 0
    if S > 1:
        epochs = (max_iter // max(1, check_every) + 3) if conv_mode == 1 else (max_iter + 2)
        ws = _coop_workspace(x.device, _stream_ptr(x), R, epochs, S)
        if coop_device_gen:
            gen = 0                         # unused: the kernel reads ws["gen_dev"]
        elif torch.cuda.is_current_stream_capturing():
            # a graph replays fixed arguments: zero this launch's granules in the graph
            # and tag them with a generation eager launches never reach
            ws["slots"][: R * epochs * S * 2].zero_()
            gen = 0xFFFFFFFF
        else:
            ws["gen"] = ws["gen"] % 0x7FFFFFFE + 1   # tags this launch's arrivals (< 2^31)
            gen = ws["gen"]
        ws_slots, ws_count, ws_flag = ws["slots"].data_ptr(), 0, ws["flag"].data_ptr()
        gen_dev = (ws["gen_dev"].data_ptr(), ws["arrive"].data_ptr()) if coop_device_gen \
            else (0, 0)
    else:
        gen = 0
        gen_dev = (0, 0)
    pl_ptr = pl_rs = pl_ld = pl_plane = pl_cols = 0
    if planes is not None:
        if (planes.dtype != torch.int16 or planes.dim() != 3
                or planes.shape[0] < min(3, int(planes_n))
                or planes.shape[1] < R * K or planes.stride(2) != 1 or planes.shape[2] < n
                or planes.device != x.device):
            raise ValueError("planes: int16 (>= planes_n, >= R*K, >= n) with unit column "
                             "stride")
        if planes_colmul is not None and (planes_colmul.dtype != torch.float32
                                          or planes_colmul.numel() < n
                                          or not planes_colmul.is_contiguous()):
            raise ValueError("planes_colmul: contiguous float32 with >= n entries")
        pl_ptr, pl_ld, pl_plane = planes.data_ptr(), planes.stride(1), planes.stride(0)
        pl_rs, pl_cols = K * pl_ld, planes.shape[2]
    gs_ptr = gs_rs = gs_ld = gs_cols = 0
    if gram is None and gram_of is not None:
        gs_ptr, gs_rs, gs_ld, gs_cols = (gram_of.data_ptr(), gram_of.stride(0),
                                         gram_of.stride(1), gram_of.shape[2])
    h.solve(a, K, x.data_ptr(), x.stride(0), x.stride(1), numer.data_ptr(), numer.stride(0),
            numer.stride(1), gram.data_ptr() if gram is not None else 0, K * K, ri, nblocks, n,
            int(max_iter), float(tol),
            float(l1_num), float(l1_den), float(l2), float(eps),
            lin_out.data_ptr() if lin_out is not None else 0,
            quad_out.data_ptr() if quad_out is not None else 0,
            iters_out.data_ptr() if iters_out is not None else 0, int(max(1, nsplit)),
            int(conv_mode), int(check_every), int(threads), vcode,
            active.data_ptr() if active is not None else 0, int(S), ws_slots, ws_count,
            int(gen), int(epochs), ws_flag, pl_ptr, int(pl_rs), int(pl_ld), int(pl_plane),
            planes_colmul.data_ptr() if (planes is not None and planes_colmul is not None) else 0,
            int(pl_cols), int(planes_n), gs_ptr, int(gs_rs), int(gs_ld), int(gs_cols),
            *f_args, *gen_dev, int(rpl), _stamp_buffer(vcode, rpl, nblocks, S, K, x),
            _stream_ptr(x))
    return int(S)


# Diagnostic phase stamps of the pipelined solve (tools/pipe_stamp_probe.py sets
# STAMPS_ON with an extension built with CNMF_PIPE_STAMPS_BUILD=1): every launch gets a
# fresh buffer, kept with its (K, slices) in STAMP_LOG for the probe.
STAMP_LOG: list = []
STAMPS_ON = False


def _stamp_buffer(vcode, rpl, nblocks, S, K, x) -> int:
    if not STAMPS_ON or vcode != 3 or torch.cuda.is_current_stream_capturing():
        return 0
    wgs = (rpl if rpl else nblocks) * max(1, int(S))
    buf = torch.zeros(wgs * 10, dtype=torch.int64, device=x.device)
    STAMP_LOG.append({"K": int(K), "S": int(S), "rounds": -(-nblocks // (rpl or nblocks)),
                      "buf": buf})
    return buf.data_ptr()


def _fused_solve_args(R, K, n, x, numer, nslabs, nstride, nscale, nbase, nout, gparts,
                      gparts_n, gout, gparts_out):
    """Validated raw arguments of the fused solve operands (see solve)."""
    if nslabs < 1 or (nslabs > 1 and nstride < 1):
        raise ValueError("numer_slabs >= 1 with a positive slab stride")
    if nslabs > 1:
        need = numer.storage_offset() + (nslabs - 1) * nstride + numer.stride(0) * (R - 1) + \
            numer.stride(1) * (K - 1) + n
        if need > numer.untyped_storage().nbytes() // 4:
            raise ValueError("numer slabs extend beyond numer's storage")
    if nscale is not None and (nscale.dtype != torch.float32 or nscale.numel() < n
                               or not nscale.is_contiguous()):
        raise ValueError("numer_scale: contiguous float32 with >= n entries")
    nb_rs = ldnb = 0
    for name, t in (("numer_base", nbase), ("numer_out", nout)):
        if t is not None:
            _check_block_view(name, t, R, K, n)
    if nbase is not None and nout is not None and nbase.stride()[:2] != nout.stride()[:2]:
        raise ValueError("numer_base and numer_out need the same strides")
    ref = nbase if nbase is not None else nout
    if ref is not None:
        nb_rs, ldnb = ref.stride(0), ref.stride(1)
    gp_rs = gp_out_rs = 0
    if gparts is not None:
        if (gparts.dim() != 4 or gparts.shape[0] < R or gparts.shape[2:] != (K, K)
                or gparts.dtype != torch.float32 or gparts.stride(3) != 1 or gparts.stride(2) != K
                or gparts.stride(1) != K * K or not 1 <= gparts_n <= gparts.shape[1]):
            raise ValueError("gram_parts: float32 (R, S, K, K) with K x K blocks contiguous")
        gp_rs = gparts.stride(0)
    if gparts_out is not None:
        if (gparts_out.dim() != 4 or gparts_out.shape[0] < R or gparts_out.shape[2:] != (K, K)
                or gparts_out.dtype != torch.float32 or gparts_out.stride(3) != 1
                or gparts_out.stride(2) != K or gparts_out.stride(1) != K * K):
            raise ValueError("gram_parts_out: float32 (R, S, K, K), K x K blocks contiguous")
        gp_out_rs = gparts_out.stride(0)
    if gout is not None and (gout.shape != (R, K, K) or not gout.is_contiguous()
                             or gout.dtype != torch.float32):
        raise ValueError("gram_out: contiguous float32 (R, K, K)")

    def ptr(t):
        return t.data_ptr() if t is not None else 0
    return (int(nslabs), int(nstride), ptr(nscale), ptr(nbase), ptr(nout), int(nb_rs), int(ldnb),
            ptr(gparts), int(gparts_n if gparts is not None else 0), int(gp_rs), ptr(gout),
            ptr(gparts_out), int(gp_out_rs))


# Cooperative-split bookkeeping.  A launch of S*nblocks 1024-thread workgroups is only safe
# (spin-waits terminate) when every workgroup is resident at once: one such workgroup per
# CU on gfx950, so the budget is the CU count minus a margin for concurrent kernels.
_COOP_WS: dict = {}
_COOP_RESIDENT: dict = {}
COOP_COLS_PER_WG = 1024
kCoopMaxSlices = 32          # solve_core.h: cooperative slices per replicate
_TLS = threading.local()


@contextlib.contextmanager
def coop_share(n: int):
    """Within this context (per host thread) cooperative solves use 1/n of the
    co-residency budget: n streams running cooperative solves at once can then never
    hold the whole chip with workgroups that wait for siblings that cannot be placed."""
    prev = getattr(_TLS, "share", 1)
    _TLS.share = max(1, int(n))
    try:
        yield
    finally:
        _TLS.share = prev


def coop_prepare(dev: torch.device) -> None:
    """Cache the device's co-residency budget (call from the thread that owns the
    device before handing work to helper threads)."""
    if dev.type == "cuda":
        _coop_resident(dev)


# CUs the cooperative solves' co-residency budget leaves to other kernels (RCCL, the
# overlapped one-shot xGMI collectives -- parallel/xgmi.py caps their blocks at this)
COOP_MARGIN_CUS = 16


def _coop_resident(dev: torch.device) -> int:
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _COOP_RESIDENT:
        # the HIP attribute, not torch.cuda.get_device_properties: its first call
        # initialises amdsmi (~26 ms inside the first factorize)
        cus = _hip.cu_count(key) if _hip is not None else \
            torch.cuda.get_device_properties(key).multi_processor_count
        _COOP_RESIDENT[key] = max(1, cus - COOP_MARGIN_CUS)
    return max(1, _COOP_RESIDENT[key] // getattr(_TLS, "share", 1))


def _coop_split(n: int, nblocks: int, dev: torch.device) -> int:
    if _ENV["CNMF_SOLVE_COOP"] == "0":
        return 1
    want = (n + COOP_COLS_PER_WG - 1) // COOP_COLS_PER_WG
    return max(1, min(want, _coop_resident(dev) // max(1, nblocks), 16))


MFMA_WG_PER_CU = 4          # solve_mfma.hip: <= 128 VGPRs and <= 37 KB LDS per workgroup


def _mfma_split(n: int, nblocks: int, K: int, nsplit: int, coop, dev: torch.device):
    """Slices per replicate for the matrix-core solve, or None when it cannot run: with
    nsplit > 1 the caller's slices must each fit a workgroup; otherwise S cooperative
    slices (all co-resident) -- at least enough for the tiles, then more while the
    budget allows so the grid fills the chip, up to ~256 columns per slice."""
    cap = _hip.solve_mfma_max_cols(K)
    if nsplit > 1:   # fixed-step column split: no cooperative slices
        return 1 if -(-n // nsplit) <= cap else None
    s_min = -(-n // cap)
    if coop != "auto":
        S = max(1, int(coop))
        return S if S >= s_min and (S == 1 or nblocks * S <= MFMA_WG_PER_CU *
                                    _coop_resident(dev)) else None
    if s_min > 1 and _ENV["CNMF_SOLVE_COOP"] == "0":
        return None
    if _ENV["CNMF_SOLVE_COOP"] == "0":
        return 1            # s_min == 1 here: one workgroup per replicate, no exchange
    budget = MFMA_WG_PER_CU * _coop_resident(dev)
    if nblocks * s_min > budget and s_min > 1:
        return None
    S = max(s_min, min(budget // max(1, nblocks), -(-n // 256), 32))
    return max(1, S)


def pipe_slices(n: int, nblocks: int, K: int, dev: torch.device) -> int | None:
    """The slice count S an unregularised block-objective MU solve of ``nblocks``
    replicates x ``n`` columns runs at under coop="auto" on the pipelined kernel (as
    ops.solve picks it), or None when that kernel does not take it."""
    if _hip is None or not _hip.solve_pipe_k(K) or _ENV["CNMF_SOLVE_PIPE"] == "0":
        return None
    S = _mfma_split(n, nblocks, K, 1, "auto", dev) if _hip.solve_mfma_max_cols(K) > 0 else None
    if S is None:
        plan = _pipe_plan(n, nblocks, K, "auto", dev)
        S = None if plan is None else plan[0]
    if S is None or S > kCoopMaxSlices or _hip.solve_pipe_tiles(K, -(-n // S)) == 0:
        return None
    return S


def pipe_round_reps(n: int, K: int, dev: torch.device) -> int:
    """How many replicates of ``n`` columns at rank K the pipelined MU solve runs in ONE
    co-resident launch round (every cooperative slice resident at once), or 0 when it
    does not take the shape.  The streaming solver sizes its live slots by this: a batch
    past it splits the usage solve into launch rounds whose lengths are each set by
    their slowest replicate."""
    if _hip is None or not _hip.solve_pipe_k(K) or n <= 0:
        return 0
    mf = _hip.solve_mfma_max_cols(K)
    cap = mf if mf > 0 else _hip.solve_pipe_max_cols(K)
    if cap <= 0:
        return 0
    s_min = -(-n // cap)
    per_cu = MFMA_WG_PER_CU if mf > 0 else _hip.solve_pipe_wg_per_cu(K)
    return max(0, per_cu * _coop_resident(dev) // s_min)


# target columns per cooperative slice of the pipelined solve (more, shorter slices fill
# the chip; fewer, longer ones wait less on each other at the exchanges).  Round 4: 256 /
# 384 / 512: K=10 13,172 / 13,229 / 13,204 rep/s, K=20 5,232 / 5,293 / 5,141 (r4i_*).
# With the single-round XCD order and the LDS-staged Grams, 17 <= K <= 32 prefers 320:
# K=20 5,601 / 5,606 vs 5,253 / 5,455 at 384, K=30 3,767 / 3,772 vs 3,760 / 3,762
# (profiles/r4zi_*)
def _pipe_slice_cols(K: int) -> int:
    # (round 6, one batch per step: K = 10 at 640 columns 14,083 / 14,149 / 14,163 against
    # 13,969 / 13,983 / 14,019 at 384 -- fewer slices wait less at the exchanges; 768
    # 14,105, 1024 13,930; K grid 21,265 vs 21,175: profiles/r6u_*, r6v_*)
    return 320 if 16 < K <= 32 else 640


def _pipe_plan(n: int, nblocks: int, K: int, coop, dev: torch.device):
    """(S, reps_per_launch) for the pipelined matrix-core solve (solve_pipe.h), or None.
    Every replicate's columns are split into S cooperative slices that each fit one
    workgroup's register tiles (S >= s_min); the launch runs the replicates in rounds of
    ``reps_per_launch`` (0: all at once) so that each round's rpl * S workgroups are
    co-resident (pipe_wg_per_cu(K) per CU).  Rounds are balanced, and S grows while the
    round's budget allows (more, shorter slices fill the chip), up to ~256 columns per
    slice."""
    cap = _hip.solve_pipe_max_cols(K)
    if cap <= 0 or nblocks <= 0:
        return None
    s_min = -(-n // cap)
    budget = _hip.solve_pipe_wg_per_cu(K) * _coop_resident(dev)
    if s_min > kCoopMaxSlices or s_min > budget:
        return None
    if s_min > 1 and _ENV["CNMF_SOLVE_COOP"] == "0":
        return None
    if coop == "auto" and _ENV["CNMF_SOLVE_COOP"] == "0":
        return 1, 0
    if coop != "auto":
        S = max(1, int(coop))
        if S < s_min or S > kCoopMaxSlices or S > budget:
            return None
        rpl = max(1, budget // S) if S > 1 else nblocks
    else:
        rounds = -(-nblocks * s_min // budget)
        rpl = -(-nblocks // rounds)
        S = max(s_min, min(budget // rpl, -(-n // _pipe_slice_cols(K)), kCoopMaxSlices))
    if S == 1:              # no cooperative exchange: residency does not matter
        return 1, 0
    return S, (rpl if rpl < nblocks else 0)


def _coop_workspace(dev: torch.device, stream: int, R: int, epochs: int, S: int) -> dict:
    """Per-(device, stream) scratch: {generation, value} granules [R*epochs*S*2] (int64,
    zeroed once at allocation; coop_sum2 in csrc/kernels/solve_core.h), the launch
    generation and the timeout flag.  Reused across launches on the same stream (stream
    order serialises); the generation only grows, so granules need no re-zeroing."""
    key = (str(dev), stream)
    ws = _COOP_WS.get(key)
    need_slots = R * epochs * S * 2
    if ws is None or ws["slots"].numel() < need_slots:
        flag = ws["flag"] if ws is not None else torch.zeros(1, dtype=torch.int32, device=dev)
        # device-side generation (solve_pipe.hip): tags from 2^31 up, never a host tag
        gen_dev = ws["gen_dev"] if ws is not None else \
            torch.full((1,), -(1 << 31), dtype=torch.int32, device=dev)
        arrive = ws["arrive"] if ws is not None else torch.zeros(1, dtype=torch.int32, device=dev)
        # a grown workspace never frees the one it replaces: HIP graphs captured earlier
        # (other layouts, other solvers -- torch hands out streams from a small pool, so
        # unrelated captures share this key) keep writing their granules there
        retired = (ws["retired"] + [ws["slots"]]) if ws is not None else []
        ws = {"slots": torch.zeros(max(need_slots, 1 << 16), dtype=torch.int64, device=dev),
              "gen": ws["gen"] if ws is not None else 0,
              "flag": flag, "gen_dev": gen_dev, "arrive": arrive, "retired": retired}
        _COOP_WS[key] = ws
    return ws


def coop_reserve(dev: torch.device, stream: int, R: int, max_iter: int, check_every: int) -> None:
    """Allocate the cooperative workspace of ``stream`` for up to R replicates x the
    epochs of a ``max_iter`` / ``check_every`` solve x the maximum slice count, NOW --
    before a HIP-graph capture on that stream, which would otherwise record the
    workspace's zero-fill (and the reset of its device-side generation) into the graph
    and replay it every time."""
    epochs = max_iter // max(1, check_every) + 3
    _coop_workspace(dev, stream, R, epochs, kCoopMaxSlices)


def coop_flags(device: torch.device | None = None) -> list:
    """[(key, flag)] of the cooperative workspaces on ``device`` (all devices if None):
    the int32 device flags a solve sets when it gave up waiting.  A caller that already
    copies results to the host packs them into that copy and hands the values to
    coop_check, instead of one synchronising read per workspace."""
    want = None
    if device is not None:
        device = torch.device(device)
        want = str(torch.device("cuda", device.index if device.index is not None
                                else torch.cuda.current_device()))
    return [(key, ws["flag"]) for key, ws in list(_COOP_WS.items())   # other threads
            if want is None or key[0] == want]                          # may add streams


def coop_check(device: torch.device | None = None, values=None, flags=None) -> None:
    """Raise if any cooperative solve on ``device`` gave up waiting (non-resident
    workgroups) -- its results would be wrong.  ``values``: the flags of ``flags`` (a
    coop_flags list) already read back by the caller; otherwise they are read here in
    one synchronising copy.  Call once per run."""
    if flags is None:
        flags = coop_flags(device)
    if not flags:
        return
    if values is None:
        values = torch.cat([f.view(-1)[:1] for _, f in flags]).cpu().tolist()
    for (key, f), v in zip(flags, values):
        if int(v):
            f.zero_()
            raise RuntimeError(f"cooperative solve failed on {key[0]} (code {int(v)}): "
                               "workgroups were not co-resident; set CNMF_SOLVE_COOP=0")


# ----------------------------------------------------------------------------- convergence
def conv_update(lin: torch.Tensor, quad: torch.Tensor, x_sq: float, state: dict, n: int,
                pass_idx: int, tol: float, final: bool, init: bool = False,
                gate: torch.Tensor | None = None, max_pass: int = 0,
                host_flags: tuple | None = None) -> None:
    """Per-replicate Frobenius error from (lin, quad) and the (prev - cur)/init < tol
    stopping rule, entirely on the device (csrc/kernels/conv.hip).  ``state`` holds
    float64 err_init/err_prev/err and int32 active/converged/n_pass tensors.
    ``pass_idx < 0`` counts passes on the device (n_pass += 1), so the launch has no
    per-pass host argument and can live in a captured graph.  ``max_pass`` > 0: a
    replicate stops after its own max_pass-th pass (replicates of a streaming batch sit
    at different passes).  ``gate`` (int32 device scalar): set to 1 while any replicate
    is active, else 0 (gemm_planes ``gate``).  ``host_flags`` (GPU): (flags, counter) --
    pinned int32 (2, >= n) and an int32 device scalar; the launch also stores the active
    flags into ``flags[counter % 2]`` through the host mapping and advances the counter,
    so the host reads a pass's flags after its event without a copy launch (the caller
    mirrors the counter: _PassPipeline)."""
    if n <= 0:
        return
    if not use_native(lin):
        reference.conv_update(lin, quad, x_sq, state, n, pass_idx, tol, final, init,
                              max_pass=max_pass)
        if gate is not None:
            gate.fill_(int(bool((state["active"][:n] != 0).any())))
        return
    hf_ptr = hc_ptr = 0
    if host_flags is not None:
        hf, hc = host_flags
        if (hf.dtype != torch.int32 or hf.dim() != 2 or hf.shape[0] != 2 or hf.shape[1] != n
                or not hf.is_pinned() or not hf.is_contiguous() or hc.dtype != torch.int32
                or hc.device != lin.device):
            raise ValueError("host_flags: (pinned contiguous int32 (2, n), int32 device scalar)")
        hf_ptr, hc_ptr = hf.data_ptr(), hc.data_ptr()
    for t in (lin, quad):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() < n:
            raise ValueError("lin/quad must be contiguous float32 with >= n entries")
    for k, dt in (("err_init", torch.float64), ("err_prev", torch.float64), ("err", torch.float64),
                  ("active", torch.int32), ("converged", torch.int32), ("n_pass", torch.int32)):
        t = state[k]
        if t.dtype != dt or not t.is_contiguous() or t.numel() < n or t.device != lin.device:
            raise ValueError(f"state[{k}] must be contiguous {dt} on {lin.device}")
    _hip.conv_update(lin.data_ptr(), quad.data_ptr(), float(x_sq), state["err_init"].data_ptr(),
                     state["err_prev"].data_ptr(), state["err"].data_ptr(),
                     state["active"].data_ptr(), state["converged"].data_ptr(),
                     state["n_pass"].data_ptr(), int(n), int(pass_idx), float(tol), int(final),
                     int(init), _gate_ptr(gate, lin.device), int(max_pass), hf_ptr, hc_ptr,
                     _stream_ptr(lin))


# ----------------------------------------------------------------------------- streaming
def stream_swap(grp: dict, ring: dict, store: dict, state: tuple, gate: torch.Tensor,
                chunks: int = 32) -> None:
    """Harvest the stopped replicates of one K group of a streaming batch into the result
    store and place the next staged replicates of its ring at their positions, on the
    device (csrc/kernels/stream.hip; NMFBatchSolver.run_stream).  ``grp``: the group's
    views -- n, K, active (n,) int32, occ (n,) int32, plan (2n,) int32, W (nK, G), HT
    (nK, N), parts (n, S, K, K), wpl (3, rows >= nK, Gp) int16; ``ring``: qc, head / tail
    (int32 device scalars), ids (qc,), W (qc K, G), HT (qc K, N), sf (3, qc) float64, si
    (5, qc) int32, parts (qc, S, K, K), wpl (3, qc K, Gp); ``store``: offs (R,) int64, W,
    HT (or None), sf (3, R), si (5, R), done (int32 scalar); ``state``: the batch's (sf,
    si) row views at the group's first position (3 / 5 rows, any row stride)."""
    n, K = int(grp["n"]), int(grp["K"])
    if n <= 0:
        return
    W, HT, rW, rHT = grp["W"], grp["HT"], ring["W"], ring["HT"]
    G, N = W.shape[1], HT.shape[1]
    sf, si = state
    wpl, rwpl = grp["wpl"], ring["wpl"]
    for name, t, dt in (("W", W, torch.float32), ("HT", HT, torch.float32),
                        ("ring W", rW, torch.float32), ("ring HT", rHT, torch.float32),
                        ("store W", store["W"], torch.float32)):
        if t.dtype != dt or t.stride(1) != 1 or t.device != W.device:
            raise ValueError(f"stream_swap: {name} must be {dt} rows with unit column stride")
    if W.shape[0] < n * K or rW.shape[0] < ring["qc"] * K or rW.stride(0) != W.stride(0) or \
            rHT.stride(0) != HT.stride(0) or store["W"].stride(0) != W.stride(0) or \
            (store["HT"] is not None and store["HT"].stride(0) != HT.stride(0)):
        raise ValueError("stream_swap: row pitches of batch, ring and store must agree")
    if wpl.shape[0] != 3 or rwpl.shape[0] != 3 or wpl.stride(1) != rwpl.stride(1) or \
            wpl.dtype != torch.int16 or rwpl.dtype != torch.int16:
        raise ValueError("stream_swap: planes must be (3, rows, Gp) int16 with one pitch")
    parts, rparts = grp["parts"], ring["parts"]
    S = parts.shape[1]
    if tuple(parts.shape[1:]) != (S, K, K) or tuple(rparts.shape[1:]) != (S, K, K) or \
            not parts.is_contiguous() or not rparts.is_contiguous():
        raise ValueError("stream_swap: contiguous (., S, K, K) partial-Gram blocks")
    for name, t, m in (("active", grp["active"], n), ("occ", grp["occ"], n),
                       ("plan", grp["plan"], 2 * n), ("ring ids", ring["ids"], ring["qc"])):
        if t.dtype != torch.int32 or not t.is_contiguous() or t.numel() < m:
            raise ValueError(f"stream_swap: {name} must be contiguous int32 (>= {m})")
    oHT = store["HT"]
    vals = [n, K, G, N, S, wpl.shape[2],
            grp["active"].data_ptr(), grp["occ"].data_ptr(), grp["plan"].data_ptr(),
            sf.data_ptr(), sf.stride(0), si.data_ptr(), si.stride(0),
            W.data_ptr(), W.stride(0), HT.data_ptr(), HT.stride(0),
            parts.data_ptr(),
            wpl.data_ptr(), wpl.stride(1), wpl.stride(0),
            int(ring["qc"]), ring["head"].data_ptr(), ring["tail"].data_ptr(),
            ring["ids"].data_ptr(), rW.data_ptr(),
            rHT.data_ptr(), ring["sf"].data_ptr(),
            ring["si"].data_ptr(), rparts.data_ptr(),
            rwpl.data_ptr(), rwpl.stride(0),
            store["offs"].data_ptr(), store["W"].data_ptr(),
            oHT.data_ptr() if oHT is not None else 0,
            store["sf"].data_ptr(), store["sf"].stride(0), store["si"].data_ptr(),
            store["si"].stride(0), store["done"].data_ptr(), gate.data_ptr()]
    if ring["sf"].stride(0) != ring["qc"] or ring["si"].stride(0) != ring["qc"]:
        raise ValueError("stream_swap: ring state rows must have stride qc")
    _hip.stream_swap(vals, int(chunks), _stream_ptr(W))


def rows_swap(pairs: torch.Tensor, K: int, mats, sf: torch.Tensor | None = None,
              si: torch.Tensor | None = None, chunks: int | None = None) -> None:
    """Exchange positions ``pairs[2i]`` <-> ``pairs[2i+1]`` in place (disjoint pairs;
    stream.hip rows_swap_kernel -- _Batch.compact's swap form): K rows per position of
    every matrix in ``mats`` (2-D float32 / int16 views with unit column stride, or 3-D
    (planes, rows, cols) int16 plane stacks) and one column of the per-position state
    tables ``sf`` (rows x R float64) / ``si`` (rows x R int32).  Only the replicates that
    change position are read or written."""
    npairs = pairs.numel() // 2
    if npairs == 0:
        return
    if pairs.dtype != torch.int32 or not pairs.is_contiguous() or pairs.numel() % 2:
        raise ValueError("rows_swap: contiguous int32 pairs [2 npairs]")
    if not use_native(pairs):
        a, b = pairs[0::2].long(), pairs[1::2].long()
        if torch.unique(torch.cat([a, b])).numel() != 2 * npairs:
            raise ValueError("rows_swap: pairs must be disjoint")
        ra = (a[:, None] * K + torch.arange(K)).reshape(-1)
        rb = (b[:, None] * K + torch.arange(K)).reshape(-1)
        for t in mats:
            t3 = t if t.dim() == 3 else t.unsqueeze(0)
            ta = t3[:, ra].clone()
            t3[:, ra] = t3[:, rb]
            t3[:, rb] = ta
        for t in (sf, si):
            if t is not None:
                ta = t[:, a].clone()
                t[:, a] = t[:, b]
                t[:, b] = ta
        return
    if len(mats) > 4:
        raise ValueError("rows_swap: at most 4 matrices")
    if chunks is None:      # ~2048 workgroups: a few pairs still spread over every CU
        chunks = max(8, min(256, 2048 // npairs))
    desc = []
    for t in mats:
        t3 = t if t.dim() == 3 else t.unsqueeze(0)
        if t3.dtype not in (torch.float32, torch.int16) or t3.stride(2) != 1 or \
                t3.device != pairs.device or t3.shape[0] > 3:
            raise ValueError("rows_swap: float32 / int16 rows with unit column stride")
        desc.append((t3.data_ptr(), t3.stride(1), t3.stride(0) if t3.shape[0] > 1 else 0,
                     t3.shape[2], t3.element_size(), t3.shape[0]))
    for name, t, dt in (("sf", sf, torch.float64), ("si", si, torch.int32)):
        if t is not None and (t.dtype != dt or t.stride(1) != 1 or t.shape[0] > 8):
            raise ValueError(f"rows_swap: {name} must be (<= 8, R) {dt} rows")
    _hip.rows_swap(pairs.data_ptr(), npairs, int(K), desc,
                   sf.data_ptr() if sf is not None else 0, sf.stride(0) if sf is not None else 0,
                   sf.shape[0] if sf is not None else 0,
                   si.data_ptr() if si is not None else 0, si.stride(0) if si is not None else 0,
                   si.shape[0] if si is not None else 0, int(chunks), _stream_ptr(pairs))


class HostMailbox:
    """Pinned host int32 rows a kernel writes directly (device-mapped pinned memory): a
    pass's small results reach the host with no copy launch.  Row s % slots holds
    [sequence number, values...]; ``read(q)`` returns pass q's values once its event
    completed (None if the row does not carry sequence q -- the caller then copies)."""

    def __init__(self, width: int, slots: int = 8):
        self.width, self.slots = int(width) + 1, int(slots)
        self.host = torch.full((self.slots, self.width), -1, dtype=torch.int32, pin_memory=True)
        self.dev_ptr = _hip.host_dev_ptr(self.host.data_ptr())

    def read(self, q: int):
        row = self.host[q % self.slots].tolist()
        return row[1:] if row[0] == q else None


def stream_publish(ctr: torch.Tensor, seq: torch.Tensor, box: HostMailbox) -> None:
    """Write the counter block ``ctr`` (int32 device) into the host mailbox row of the
    device sequence counter ``seq`` (int32 device scalar, advanced) -- stream.hip."""
    if ctr.dtype != torch.int32 or not ctr.is_contiguous() or seq.dtype != torch.int32:
        raise ValueError("stream_publish: contiguous int32 counters and sequence")
    _hip.stream_publish(ctr.data_ptr(), ctr.numel(), seq.data_ptr(), box.dev_ptr, box.slots,
                        box.width, _stream_ptr(ctr))


# ----------------------------------------------------------------------------- beta MU
def beta_mode(beta: float) -> int:
    return 0 if beta == 1.0 else (1 if beta == 0.0 else 2)


BP_KL_FP16, BP_KL = 0, 3


def bp_mode(beta: float) -> int:
    """Mode of the split-bf16 beta kernels (beta_planes.h BpMode): KL runs the
    fp32-accurate numerator (kBpKLX = 3: Q = X / P in two bf16 planes, S in two -- <= 3 *
    2^-16 relative per term, random sign, inside the fp32 accumulation error of the
    reduction, as the reference's fp32 nmf-torch run) unless ``CNMF_KL_FP16=1`` selects the
    faster fp16 numerator (kBpKL = 0: <= 2^-11 per term); IS 1, other beta 2."""
    m = beta_mode(beta)
    if m == 0 and _ENV["CNMF_KL_FP16"] != "1":
        return BP_KL
    return m


def _bp_kl(mode: int) -> bool:
    return mode in (BP_KL_FP16, BP_KL)


def beta_contract(side: str, X: torch.Tensor, HT3: torch.Tensor, W3: torch.Tensor,
                  beta: float, eps: float, want_num: bool = True, want_loss: bool = False,
                  active: torch.Tensor | None = None, splits: int | None = None,
                  reduce: bool = True):
    """Fused beta-divergence MU contraction (csrc/kernels/beta_mu.hip).

    ``X`` (N, G) with unit column stride; ``HT3`` (R, K, N) and ``W3`` (R, K, G) views with
    unit inner stride.  With P = max(HT^T W, eps), Q = X P^(beta-2), D = P^(beta-1):
      side "h": num = W Q^T (R,K,N), den = W D^T (None when beta == 1: den is rowsum W)
      side "w": num = HT Q  (R,K,G), den = HT D  (None when beta == 1: den is rowsum HT)
    ``want_loss`` (side "h") also returns sum D_beta(X || P) per replicate (float64).
    Replicates whose ``active`` flag is 0 are skipped (their outputs are unspecified).
    ``reduce=False`` (side "w") returns num/den as (splits, R, K, G) partials, the operand
    layout of :func:`beta_w_update` (which sums them itself).
    """
    s = {"h": 0, "w": 1}[side]
    R, K, N = HT3.shape
    G = W3.shape[2]
    if X.shape != (N, G) or W3.shape[:2] != (R, K):
        raise ValueError(f"beta_contract: X {tuple(X.shape)}, HT3 {tuple(HT3.shape)}, "
                         f"W3 {tuple(W3.shape)} are inconsistent")
    if not use_native(HT3):
        num, den, loss = reference.beta_contract(s, X, HT3, W3, beta, eps, want_num, want_loss,
                                                 active)
        if not reduce and num is not None:
            num = num.unsqueeze(0)
            den = den.unsqueeze(0) if den is not None else None
        return num, den, loss
    if beta_any_k(K, beta):
        num, den, loss = _beta_contract_any(s, X, HT3, W3, beta, eps, want_num, want_loss,
                                            active)
        if not reduce and num is not None:
            num = num.unsqueeze(0)
            den = den.unsqueeze(0) if den is not None else None
        return num, den, loss
    _native_dtype_k("beta_contract", HT3.dtype, K, _hip.beta_max_k())
    for name, t in (("X", X), ("HT3", HT3), ("W3", W3)):
        if t.dtype != torch.float32 or t.device != HT3.device:
            raise ValueError(f"{name}: float32 on {HT3.device} required")
        if t.stride(-1) != 1:
            raise ValueError(f"{name}: unit inner stride required, got {t.stride()}")
    if active is not None and (active.dtype != torch.int32 or active.numel() < R
                               or not active.is_contiguous()):
        raise ValueError("active: contiguous int32 with >= R entries")
    if s == 1 and not want_num:
        raise ValueError("side 'w' computes the numerator")
    mode = beta_mode(beta)
    dev = HT3.device
    if s == 0:
        out_shape = (R, K, N)
        n_split = 1
    else:
        out_shape = (R, K, G)
        if splits is None:
            units = ((G + 63) // 64) * R
            n_split = max(1, min(64, -(-2048 // max(1, units)), N // 1024 or 1))
        else:
            n_split = max(1, int(splits))
    num = den = loss = None
    if want_num:
        num = torch.empty((n_split,) + out_shape, device=dev, dtype=torch.float32)
        if mode != 0:
            den = torch.empty_like(num)
    n_strips = (N + 63) // 64
    if want_loss and s == 0:
        loss = torch.zeros((R, n_strips), device=dev, dtype=torch.float64)
    _hip.beta_contract(s, mode, X.data_ptr(), X.stride(0), HT3.data_ptr(), HT3.stride(0),
                       HT3.stride(1), W3.data_ptr(), W3.stride(0), W3.stride(1), N, G, K, R,
                       float(beta), float(eps), num.data_ptr() if num is not None else 0,
                       den.data_ptr() if den is not None else 0,
                       loss.data_ptr() if loss is not None else 0,
                       active.data_ptr() if active is not None else 0, n_split, 0, 0, 0.0, 0.0,
                       1.0, 0.0, 0, 0, 0, 0, 0, 1, 0, _stream_ptr(HT3))
    if num is not None and not reduce:
        return num, den, None
    if num is not None:
        num = num[0] if n_split == 1 else num.sum(0)
        if den is not None:
            den = den[0] if n_split == 1 else den.sum(0)
    if loss is not None:
        loss = loss.sum(1)
    return num, den, loss


_BETA_WS: dict = {}


def beta_update_h(X: torch.Tensor, HT3: torch.Tensor, W3: torch.Tensor, beta: float, eps: float,
                  l1: float = 0.0, l2: float = 0.0, gamma: float = 1.0,
                  act: torch.Tensor | None = None, tol: float | None = None,
                  iters: torch.Tensor | None = None,
                  den_vec: torch.Tensor | None = None, conv_mode: int = 0,
                  check_every: int = 10, hstate: torch.Tensor | None = None) -> None:
    """One fused in-place beta-MU step of the usages: HT3 *= (num/(den+l1+l2 HT3))^gamma
    with num/den from the H-side contraction -- the numerator never leaves registers.

    ``act`` (int32 (R,), optional) gates replicates; with ``tol`` the kernel also applies
    the inner stopping rule on device: act[r] = 0 once ||dh||/(||h||+eps) < tol, and
    iters[r] += 1 for every replicate that stepped.  ``den_vec`` (KL only): the row sums
    of W3 as contiguous float32 (R, K) -- pass it when W3 is fixed across many steps.
    ``conv_mode`` 1 replaces the iterate-change rule by the block objective: the chunk's
    beta-divergence (of the usages BEFORE the step) is recorded every ``check_every``
    steps in ``hstate`` (float64 (R, 2): last objective, steps; zero it before a solve)
    and a replicate stops after a step where it changed by <= tol relative."""
    R, K, N = HT3.shape
    G = W3.shape[2]
    if tol is not None and conv_mode == 1 and (
            hstate is None or hstate.dtype != torch.float64 or hstate.numel() < 2 * R
            or not hstate.is_contiguous() or hstate.device != HT3.device):
        raise ValueError("conv_mode 1 needs hstate: contiguous float64 (R, 2) on the device")
    if not use_native(HT3):
        return reference.beta_update_h(X, HT3, W3, beta, eps, l1, l2, gamma, act, tol, iters,
                                       conv_mode, check_every, hstate)
    if beta_any_k(K, beta):
        return reference.beta_update_h(X, HT3, W3, beta, eps, l1, l2, gamma, act, tol, iters,
                                       conv_mode, check_every, hstate,
                                       contract=_beta_contract_any)
    _native_dtype_k("beta_update_h", HT3.dtype, K, _hip.beta_max_k())
    if X.shape != (N, G) or W3.shape[:2] != (R, K):
        raise ValueError("beta_update_h: inconsistent shapes")
    for name, t in (("X", X), ("HT3", HT3), ("W3", W3)):
        if t.dtype != torch.float32 or t.device != HT3.device or t.stride(-1) != 1:
            raise ValueError(f"{name}: float32, unit inner stride, on {HT3.device} required")
    for name, t in (("act", act), ("iters", iters)):
        if t is not None and (t.dtype != torch.int32 or t.numel() < R or not t.is_contiguous()):
            raise ValueError(f"{name}: contiguous int32 with >= R entries")
    if tol is not None and act is None:
        raise ValueError("the inner stopping rule needs an act array")
    mode = beta_mode(beta)
    dev = HT3.device
    if mode != 0:
        den_vec = None
    elif den_vec is None:
        den_vec = W3.sum(dim=2, dtype=torch.float32).contiguous()
    elif (den_vec.shape != (R, K) or den_vec.dtype != torch.float32
          or not den_vec.is_contiguous() or den_vec.device != dev):
        raise ValueError("den_vec: contiguous float32 (R, K) on the device required")
    n_strips = (N + 63) // 64
    part = counter = None
    if tol is not None:
        key = (str(dev), _stream_ptr(HT3))
        ws = _BETA_WS.get(key)
        if ws is None or ws["part"].numel() < R * n_strips * 3 or ws["counter"].numel() < R:
            ws = {"part": torch.empty(max(R * n_strips * 3, 1 << 12), device=dev),
                  "counter": torch.zeros(max(R, 1024), dtype=torch.int32, device=dev)}
            _BETA_WS[key] = ws
        part, counter = ws["part"], ws["counter"]
    _hip.beta_contract(0, mode, X.data_ptr(), X.stride(0), HT3.data_ptr(), HT3.stride(0),
                       HT3.stride(1), W3.data_ptr(), W3.stride(0), W3.stride(1), N, G, K, R,
                       float(beta), float(eps), 0, 0, 0,
                       act.data_ptr() if act is not None else 0, 1, 1,
                       den_vec.data_ptr() if den_vec is not None else 0, float(l1), float(l2),
                       float(gamma), float(tol if tol is not None else 0.0),
                       part.data_ptr() if part is not None else 0,
                       counter.data_ptr() if counter is not None else 0,
                       act.data_ptr() if (act is not None and tol is not None) else 0,
                       iters.data_ptr() if (iters is not None and tol is not None) else 0,
                       int(conv_mode), int(check_every),
                       hstate.data_ptr() if (hstate is not None and tol is not None) else 0,
                       _stream_ptr(HT3))


def beta_w_update(W3: torch.Tensor, num: torch.Tensor, den: torch.Tensor | None,
                  hsum: torch.Tensor | None, An: torch.Tensor, Ad: torch.Tensor,
                  an_out: torch.Tensor, dn_out: torch.Tensor | None, beta: float, gamma: float,
                  l1: float, l2: float, eps: float, tol: float, act: torch.Tensor,
                  iters: torch.Tensor | None = None) -> None:
    """One anchored online beta-MU step of the spectra, in place (beta_mu.hip
    beta_w_update_kernel):  an = W^(1/gamma) num,  W <- ((An + an) / (Ad + den + l1 +
    l2 W))^gamma, with num/den the (splits, R, K, G) partials of the chunk's W-side
    contraction at the current W (den None for KL, whose denominator is ``hsum`` (R, K),
    the chunk's usage sums; ``Ad`` is then (R, K)).  ``an_out``/``dn_out`` receive the
    step's anchored statistics.  Replicates with act == 0 are untouched; the others stop
    (act -> 0) once |dW| / (|W| + eps) < tol, and count the step in ``iters``."""
    R, K, G = W3.shape
    kl = beta == 1.0
    if not use_native(W3):
        return reference.beta_w_update(W3, num, den, hsum, An, Ad, an_out, dn_out, beta, gamma,
                                       l1, l2, eps, tol, act, iters)
    _native_dtype_k("beta_w_update", W3.dtype, K, 1 << 30)
    splits = num.shape[0]
    want = {"num": (num, (splits, R, K, G)), "An": (An, (R, K, G)), "an_out": (an_out, (R, K, G)),
            "Ad": (Ad, (R, K) if kl else (R, K, G))}
    if kl:
        want["hsum"] = (hsum, (R, K))
    else:
        want["den"] = (den, (splits, R, K, G))
        want["dn_out"] = (dn_out, (R, K, G))
    for name, (t, shp) in want.items():
        if (t is None or tuple(t.shape) != shp or t.dtype != torch.float32
                or not t.is_contiguous() or t.device != W3.device):
            raise ValueError(f"beta_w_update: {name} must be contiguous float32 {shp}")
    if W3.stride(2) != 1:
        raise ValueError("beta_w_update: W3 needs unit inner stride")
    for name, t in (("act", act), ("iters", iters)):
        if t is not None and (t.dtype != torch.int32 or t.numel() < R or not t.is_contiguous()):
            raise ValueError(f"{name}: contiguous int32 with >= R entries")
    nb = int(_hip.beta_w_update_blocks(K, G))
    key = (str(W3.device), _stream_ptr(W3), "w")
    ws = _BETA_WS.get(key)
    if ws is None or ws["part"].numel() < R * nb * 2 or ws["counter"].numel() < R:
        ws = {"part": torch.empty(max(R * nb * 2, 1 << 12), device=W3.device),
              "counter": torch.zeros(max(R, 1024), dtype=torch.int32, device=W3.device)}
        _BETA_WS[key] = ws
    _hip.beta_w_update(beta_mode(beta), W3.data_ptr(), W3.stride(0), W3.stride(1),
                       num.data_ptr(), den.data_ptr() if den is not None else 0,
                       hsum.data_ptr() if hsum is not None else 0, An.data_ptr(), Ad.data_ptr(),
                       an_out.data_ptr(), dn_out.data_ptr() if dn_out is not None else 0,
                       R, K, G, splits, float(gamma), float(l1), float(l2), float(eps),
                       float(tol), ws["part"].data_ptr(), ws["counter"].data_ptr(),
                       act.data_ptr(), iters.data_ptr() if iters is not None else 0,
                       _stream_ptr(W3))


# ------------------------------------------------------- beta MU on split bf16 planes
_BP_WS: dict = {}


def _bp_ws(dev, stream, R: int, n_strips: int) -> dict:
    key = (str(dev), stream)
    ws = _BP_WS.get(key)
    if ws is None or ws["part"].numel() < R * n_strips * 4 or ws["counter"].numel() < R:
        ws = {"part": torch.empty(max(R * n_strips * 4, 1 << 12), dtype=torch.float64,
                                  device=dev),
              "counter": torch.zeros(max(R, 1024), dtype=torch.int32, device=dev)}
        _BP_WS[key] = ws
    return ws


def _bp_check(name: str, t: torch.Tensor, dev) -> None:
    if t.dtype != torch.float32 or t.device != dev or t.stride(-1) != 1:
        raise ValueError(f"{name}: float32 with unit inner stride on {dev} required, got "
                         f"{t.dtype} {tuple(t.stride())} on {t.device}")


def beta_panels(F3: torch.Tensor, beta: float, out: torch.Tensor | None = None,
                row_scale: torch.Tensor | None = None) -> torch.Tensor:
    """Split operand panels of F3 (R, K, L), unit inner stride, K <= 32, for the beta-MU
    kernels at ``beta`` (beta_planes.hip bp_panel_kernel): per replicate, chunks of 64 rows
    of the L axis, each holding the bf16 planes of the P-product layout (6 terms; KL 3) and
    the two planes of the permuted numerator layout (KL: fp16, row-scaled, with the scales
    in a tail).  ``row_scale`` (L,) float32 (KL only): the P-product panel is built from
    F[k][l] * row_scale[l] -- the usage-side panels for fp16 count X (x = c u_l, row_scale
    = 1 / u, so c / P' = x / P; :func:`beta_h_block` ``xh``).  Returns (R, panel_elems)
    int16."""
    R, K, L = F3.shape
    if use_native(F3) and beta_any_k(K, beta):
        # the rank-general path reads F3 itself (an empty placeholder keeps callers uniform)
        return torch.empty((R, 0), dtype=torch.int16, device=F3.device)
    _native_dtype_k("beta_panels", F3.dtype, K, _hip.bp_max_k())
    _bp_check("F3", F3, F3.device)
    mode = bp_mode(beta)
    if row_scale is not None and (mode != BP_KL_FP16 or row_scale.dtype != torch.float32
                                  or row_scale.numel() < L or not row_scale.is_contiguous()
                                  or row_scale.device != F3.device):
        raise ValueError("row_scale: fp16 KL (CNMF_KL_FP16=1) only, contiguous float32 (L,) "
                         "on the device")
    n = int(_hip.bp_panel_elems(K, L, mode))
    if out is None or out.shape != (R, n) or out.dtype != torch.int16 or not out.is_contiguous():
        out = torch.empty((R, n), dtype=torch.int16, device=F3.device)
    _hip.bp_panels(F3.data_ptr(), F3.stride(0), F3.stride(1), K, L, R, mode,
                   row_scale.data_ptr() if row_scale is not None else 0, out.data_ptr(), n,
                   _stream_ptr(F3))
    out._cnmf_row_scaled = row_scale is not None
    return out


def _bp_panels_check(panels: torch.Tensor, R: int, K: int, L: int, mode: int) -> None:
    n = int(_hip.bp_panel_elems(K, L, mode))
    if (panels.dim() != 2 or panels.shape[0] < R or panels.shape[1] != n
            or panels.dtype != torch.int16 or panels.stride(1) != 1):
        raise ValueError(f"panels: int16 (R, {n}) for K={K}, L={L}, beta mode {mode} required "
                         f"(beta_panels with the same beta), got {tuple(panels.shape)}")


def beta_h_block(X: torch.Tensor, HT3: torch.Tensor, W3: torch.Tensor, beta: float, eps: float,
                 nsteps: int, l1: float = 0.0, l2: float = 0.0, gamma: float = 1.0,
                 act: torch.Tensor | None = None, tol: float | None = None,
                 iters: torch.Tensor | None = None, conv_mode: int = 1,
                 hstate: torch.Tensor | None = None, loss_entry: bool = False,
                 den_vec: torch.Tensor | None = None,
                 panels: torch.Tensor | None = None, xsum: float | None = None,
                 xh: torch.Tensor | None = None, unit: torch.Tensor | None = None) -> None:
    """``nsteps`` fused beta-MU steps of the usages HT3 (R, K, N) in place against the
    spectra W3 (R, K, G) on rows X (N, G), in ONE launch (beta_planes.hip, side 0):
    HT3 *= (num / (den + l1 + l2 HT3))^gamma with num/den of the split-bf16 MFMA
    contraction.  With ``tol`` the stopping rule runs on the device after the block:
    conv_mode 1 -- the block objective D_beta(X | HT3^T W3) at the iterate the block's last
    step starts from (read off that step's own P pass; after the block when nsteps == 1)
    against the previous one (``loss_entry``: the objective before the block, computed in
    this launch; else the value ``hstate`` (float64 (R, 2): last objective, checks) holds);
    conv_mode 0 -- relative change of the last step.  act[r] -> 0 when the rule holds; iters[r] += nsteps.  ``panels``: the
    :func:`beta_panels` of W3 (built here when omitted); ``xsum``: sum(X) in float64 (KL
    objective; computed here -- one host sync -- when omitted).  KL on fp16 counts: ``xh``
    (N, G) float16 with X == xh * ``unit`` (per gene) is read instead of X (half the
    bytes; X itself is only used for shapes), with ``panels`` built by
    :func:`beta_panels` with ``row_scale = 1 / unit``."""
    R, K, N = HT3.shape
    G = W3.shape[2]
    if X.shape != (N, G) or W3.shape[:2] != (R, K):
        raise ValueError(f"beta_h_block: X {tuple(X.shape)}, HT3 {tuple(HT3.shape)}, "
                         f"W3 {tuple(W3.shape)} are inconsistent")
    if tol is not None and act is None:
        raise ValueError("the stopping rule needs an act array")
    if tol is not None and conv_mode == 1 and (
            hstate is None or hstate.dtype != torch.float64 or hstate.numel() < 2 * R
            or not hstate.is_contiguous() or hstate.device != HT3.device):
        raise ValueError("conv_mode 1 needs hstate: contiguous float64 (R, 2) on the device")
    if not use_native(HT3):
        return reference.beta_h_block(X, HT3, W3, beta, eps, nsteps, l1, l2, gamma, act, tol,
                                      iters, conv_mode, hstate, loss_entry)
    if beta_any_k(K, beta):
        return reference.beta_h_block(X, HT3, W3, beta, eps, nsteps, l1, l2, gamma, act, tol,
                                      iters, conv_mode, hstate, loss_entry,
                                      contract=_beta_contract_any)
    dev = HT3.device
    _native_dtype_k("beta_h_block", HT3.dtype, K, _hip.bp_max_k())
    for name, t in (("X", X), ("HT3", HT3), ("W3", W3)):
        _bp_check(name, t, dev)
    for name, t in (("act", act), ("iters", iters)):
        if t is not None and (t.dtype != torch.int32 or t.numel() < R or not t.is_contiguous()):
            raise ValueError(f"{name}: contiguous int32 with >= R entries")
    mode = bp_mode(beta)
    rule_loss = tol is not None and conv_mode == 1
    if _bp_kl(mode) and (nsteps > 0 or rule_loss):
        if den_vec is None:
            den_vec = W3.sum(dim=2, dtype=torch.float32).contiguous()
        elif (den_vec.shape != (R, K) or den_vec.dtype != torch.float32
              or not den_vec.is_contiguous() or den_vec.device != dev):
            raise ValueError("den_vec: contiguous float32 (R, K) on the device required")
    else:
        den_vec = None
    if xh is not None:
        if (mode != BP_KL_FP16 or xh.dtype != torch.float16 or xh.shape != (N, G) or xh.stride(1) != 1
                or unit is None or unit.numel() < G or unit.dtype != torch.float32):
            raise ValueError("xh: KL, float16 (N, G) counts with a float32 (G,) unit")
        if panels is None or not getattr(panels, "_cnmf_row_scaled", False):
            raise ValueError("xh needs panels built with row_scale = 1 / unit")
    if panels is None:
        panels = beta_panels(W3, beta)
    _bp_panels_check(panels, R, K, G, mode)
    if xh is None and getattr(panels, "_cnmf_row_scaled", False):
        raise ValueError("row-scaled panels (fp16 counts) need xh")
    n_strips = -(-N // int(_hip.bp_strip_cols(K, mode)))
    part = counter = 0
    if tol is not None:
        ws = _bp_ws(dev, _stream_ptr(HT3), R, n_strips)
        part, counter = ws["part"].data_ptr(), ws["counter"].data_ptr()
    xs = xh if xh is not None else X
    _hip.bp_run(0, mode, xs.data_ptr(), xs.stride(0), panels.data_ptr(), panels.stride(0),
                HT3.data_ptr(), HT3.stride(0), HT3.stride(1), K, N, G, R, 1, float(beta),
                float(eps), 0, 0, int(nsteps), int(bool(loss_entry) and tol is not None),
                int(tol is not None and conv_mode == 1),
                den_vec.data_ptr() if den_vec is not None else 0, float(l1), float(l2),
                float(gamma), float(tol if tol is not None else 0.0), int(conv_mode),
                hstate.data_ptr() if (hstate is not None and tol is not None) else 0,
                part, counter, act.data_ptr() if act is not None else 0,
                iters.data_ptr() if (iters is not None and tol is not None) else 0,
                act.data_ptr() if act is not None else 0, 0,
                float(xsum if xsum is not None else (
                    float(X.sum(dtype=torch.float64)) if (_bp_kl(mode) and rule_loss) else 0.0)),
                int(xh is not None), unit.data_ptr() if xh is not None else 0, 0,
                _stream_ptr(HT3))


def beta_loss(X: torch.Tensor, HT3: torch.Tensor, W3: torch.Tensor, beta: float, eps: float,
              active: torch.Tensor | None = None,
              panels: torch.Tensor | None = None) -> torch.Tensor:
    """sum D_beta(X || HT3^T W3) per replicate, float64 (R,) on the device (beta_planes.hip
    side 0 in loss-only mode: the P contraction and the loss terms, no numerator)."""
    R, K, N = HT3.shape
    G = W3.shape[2]
    if X.shape != (N, G) or W3.shape[:2] != (R, K):
        raise ValueError("beta_loss: inconsistent shapes")
    if not use_native(HT3):
        return reference.beta_contract(0, X, HT3, W3, beta, eps, False, True, active)[2]
    if beta_any_k(K, beta):
        return _beta_contract_any(0, X, HT3, W3, beta, eps, False, True, active)[2]
    dev = HT3.device
    _native_dtype_k("beta_loss", HT3.dtype, K, _hip.bp_max_k())
    for name, t in (("X", X), ("HT3", HT3), ("W3", W3)):
        _bp_check(name, t, dev)
    if active is not None and (active.dtype != torch.int32 or active.numel() < R
                               or not active.is_contiguous()):
        raise ValueError("active: contiguous int32 with >= R entries")
    mode = bp_mode(beta)
    if panels is None:
        panels = beta_panels(W3, beta)
    _bp_panels_check(panels, R, K, G, mode)
    # KL: the kernel sums x log(x/p) + p; the -sum(x) term is added here on the device
    wsum = W3.sum(dim=2, dtype=torch.float32).contiguous() if _bp_kl(mode) else None
    n_strips = -(-N // int(_hip.bp_strip_cols(K, mode)))
    loss = torch.zeros((R, n_strips), dtype=torch.float64, device=dev)
    _hip.bp_run(0, mode, X.data_ptr(), X.stride(0), panels.data_ptr(),
                panels.stride(0), HT3.data_ptr(), HT3.stride(0), HT3.stride(1), K, N, G, R, 1,
                float(beta), float(eps), 0, 0, 0, 0, 1,
                wsum.data_ptr() if wsum is not None else 0, 0.0, 0.0, 1.0, 0.0, 0, 0, 0, 0, 0,
                0, active.data_ptr() if active is not None else 0, loss.data_ptr(), 0.0,
                0, 0, 0, _stream_ptr(HT3))
    tot = loss.sum(1)
    if _bp_kl(mode):
        tot = tot - X.sum(dtype=torch.float64)
    return tot


def beta_w_partials(X: torch.Tensor, XT: torch.Tensor | None, HT3: torch.Tensor,
                    W3: torch.Tensor, beta: float, eps: float,
                    active: torch.Tensor | None = None, splits: int | None = None,
                    panels: torch.Tensor | None = None, xth: torch.Tensor | None = None,
                    unit_inv: torch.Tensor | None = None):
    """W-side beta-MU statistics of rows X (c, G) with the chunk's usages HT3 (R, K, c):
    num = HT Q, den = HT D (None for KL) as (splits, R, K, G) partials -- the operand
    layout of :func:`beta_w_update` (beta_planes.hip side 1: HT streamed from its split-bf16
    panels, W3 the fixed operand, X read through its transpose ``XT`` (G, c)).  KL on fp16
    counts: ``xth`` (G, c) float16 with X^T == xth * unit per row, ``unit_inv`` = 1 / unit
    (G,) -- read instead of XT (which may then be None)."""
    R, K, c = HT3.shape
    G = W3.shape[2]
    if X.shape != (c, G) or W3.shape[:2] != (R, K):
        raise ValueError("beta_w_partials: inconsistent shapes")
    if not use_native(HT3):
        num, den, _ = reference.beta_contract(1, X, HT3, W3, beta, eps, True, False, active)
        return num.unsqueeze(0), (den.unsqueeze(0) if den is not None else None)
    if beta_any_k(K, beta):
        num, den, _ = _beta_contract_any(1, X, HT3, W3, beta, eps, True, False, active)
        return num.unsqueeze(0), (den.unsqueeze(0) if den is not None else None)
    dev = HT3.device
    _native_dtype_k("beta_w_partials", HT3.dtype, K, _hip.bp_max_k())
    if xth is not None:
        if (beta_mode(beta) != 0 or xth.dtype != torch.float16 or xth.shape != (G, c)
                or xth.stride(1) != 1 or unit_inv is None or unit_inv.numel() < G
                or unit_inv.dtype != torch.float32):
            raise ValueError("xth: KL, float16 (G, c) counts with a float32 (G,) unit_inv")
    elif XT is None or XT.shape != (G, c):
        raise ValueError("beta_w_partials: XT (G, c) required on the device")
    for name, t in (("HT3", HT3), ("W3", W3)) + ((("XT", XT),) if xth is None else ()):
        _bp_check(name, t, dev)
    if active is not None and (active.dtype != torch.int32 or active.numel() < R
                               or not active.is_contiguous()):
        raise ValueError("active: contiguous int32 with >= R entries")
    mode = bp_mode(beta)
    if panels is None:
        panels = beta_panels(HT3, beta)
    _bp_panels_check(panels, R, K, c, mode)
    if splits is None:
        units = -(-G // int(_hip.bp_strip_cols(K, mode))) * R
        splits = max(1, min(16, -(-2048 // max(1, units))))
    n_split = int(_hip.bp_splits(c, int(splits)))
    num = torch.empty((n_split, R, K, G), dtype=torch.float32, device=dev)
    den = torch.empty_like(num) if not _bp_kl(mode) else None
    xs = xth if xth is not None else XT
    _hip.bp_run(1, mode, xs.data_ptr(), xs.stride(0), panels.data_ptr(), panels.stride(0),
                W3.data_ptr(), W3.stride(0), W3.stride(1), K, G, c, R, n_split, float(beta),
                float(eps), num.data_ptr(), den.data_ptr() if den is not None else 0, 1, 0, 0,
                0, 0.0, 0.0, 1.0, 0.0, 0, 0, 0, 0, 0, 0,
                active.data_ptr() if active is not None else 0, 0, 0.0, int(xth is not None), 0,
                unit_inv.data_ptr() if xth is not None else 0, _stream_ptr(HT3))
    return num, den


# ------------------------------------------------------------- sparse KL (CSR X)
class KLCSR(NamedTuple):
    """CSR of a non-negative matrix for the sparse KL kernels (sparse_kl.hip): row i owns
    entries [rowptr[i], rowptr[i+1]) of col / val; a row range is a rowptr slice over the
    same col / val (:func:`kl_csr_rows`)."""
    rowptr: torch.Tensor    # int32 (n_rows + 1,), absolute offsets
    col: torch.Tensor       # int32
    val: torch.Tensor       # float32
    n_rows: int
    n_cols: int


def kl_csr(X: torch.Tensor) -> KLCSR:
    """CSR (x != 0 entries, row-major) of a dense float32 matrix on the device (one
    nonzero() host sync)."""
    n, m = X.shape
    rows, cols = torch.nonzero(X, as_tuple=True)
    rowptr = torch.zeros(n + 1, dtype=torch.int64, device=X.device)
    rowptr[1:] = torch.bincount(rows, minlength=n).cumsum(0)
    return KLCSR(rowptr.to(torch.int32), cols.to(torch.int32).contiguous(),
                 X[rows, cols].to(torch.float32).contiguous(), n, m)


def kl_csr_rows(csr: KLCSR, a: int, b: int) -> KLCSR:
    return KLCSR(csr.rowptr[a:b + 1], csr.col, csr.val, b - a, csr.n_cols)


def kl_tile_rows(K: int) -> int:
    """Streamed rows per LDS tile of the sparse KL kernels (S^T staged in 128 KB)."""
    return (128 * 1024 // (4 * int(_hip.sk_k4(K)))) // 64 * 64


def kl_csr_tiles(Xc: torch.Tensor, K: int) -> list:
    """The spectra-side CSRs of a row chunk Xc (c, G): [(t0, CSR of Xc[t0:t1]^T)] over
    tiles of :func:`kl_tile_rows` cells, each sized to have its usages staged in LDS."""
    c = Xc.shape[0]
    tl = kl_tile_rows(K)
    return [(t0, kl_csr(Xc[t0:min(c, t0 + tl)].t())) for t0 in range(0, c, tl)]


def kl_st(F3: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """(R, L, K4) transpose of F3 (R, K, L), rows zero-padded to K4 = 4 ceil(K / 4) (the
    sparse KL kernels gather one float4-aligned row per non-zero)."""
    R, K, L = F3.shape
    K4 = int(_hip.sk_k4(K))
    if out is None or out.shape != (R, L, K4) or not out.is_contiguous():
        out = torch.zeros((R, L, K4), dtype=torch.float32, device=F3.device)
    out[:, :, :K].copy_(F3.transpose(1, 2))
    return out


def _sk_args(csr: KLCSR, F3: torch.Tensor, S3: torch.Tensor, st: torch.Tensor | None):
    R, K, Lf = F3.shape
    Ls = S3.shape[2]
    if csr.n_rows != Lf or csr.n_cols != Ls or csr.rowptr.dtype != torch.int32:
        raise ValueError(f"CSR {csr.n_rows} x {csr.n_cols} does not match fixed {Lf} x "
                         f"streamed {Ls}")
    _native_dtype_k("sparse KL", F3.dtype, K, 32)
    for name, t in (("F3", F3), ("S3", S3)):
        _bp_check(name, t, F3.device)
    if st is None:
        st = kl_st(S3)
    if (st.shape != (R, Ls, int(_hip.sk_k4(K))) or st.stride(2) != 1
            or st.stride(1) != st.shape[2] or st.data_ptr() % 16):
        raise ValueError("st: kl_st(S3) (or a row range of it) required")
    return st


def kl_sparse_h_block(csr: KLCSR, HT3: torch.Tensor, W3: torch.Tensor, eps: float,
                      nsteps: int, l1: float = 0.0, l2: float = 0.0,
                      act: torch.Tensor | None = None, tol: float | None = None,
                      iters: torch.Tensor | None = None, conv_mode: int = 1,
                      hstate: torch.Tensor | None = None, loss_entry: bool = False,
                      den_vec: torch.Tensor | None = None, st: torch.Tensor | None = None,
                      xsum: float | None = None) -> None:
    """:func:`beta_h_block` at beta = 1 over the CSR rows ``csr`` (cells x genes) of X:
    ``nsteps`` fused KL MU steps of HT3 (R, K, c) in place against W3 (R, K, G), the same
    on-device stopping rule (sparse_kl.hip side 0).  ``st``: :func:`kl_st` of W3."""
    R, K, N = HT3.shape
    if tol is not None and act is None:
        raise ValueError("the stopping rule needs an act array")
    if tol is not None and conv_mode == 1 and (
            hstate is None or hstate.dtype != torch.float64 or hstate.numel() < 2 * R):
        raise ValueError("conv_mode 1 needs hstate: contiguous float64 (R, 2)")
    _require_native()
    st = _sk_args(csr, HT3, W3, st)
    if den_vec is None:
        den_vec = W3.sum(dim=2, dtype=torch.float32).contiguous()
    part = counter = 0
    if tol is not None:
        ws = _bp_ws(HT3.device, _stream_ptr(HT3), R, int(_hip.sk_groups(N, R, W3.shape[2], K)))
        part, counter = ws["part"].data_ptr(), ws["counter"].data_ptr()
    rule_loss = tol is not None and conv_mode == 1
    if rule_loss and xsum is None:
        xsum = float(csr.val[int(csr.rowptr[0]):int(csr.rowptr[-1])].sum(dtype=torch.float64))
    _hip.sk_run(0, csr.rowptr.data_ptr(), csr.col.data_ptr(), csr.val.data_ptr(), st.data_ptr(),
                st.stride(0), HT3.data_ptr(), HT3.stride(0), HT3.stride(1), K, N, W3.shape[2], R,
                float(eps),
                0, int(nsteps), int(bool(loss_entry) and tol is not None), int(rule_loss),
                den_vec.data_ptr(), float(l1), float(l2),
                float(tol if tol is not None else 0.0), int(conv_mode),
                hstate.data_ptr() if (hstate is not None and tol is not None) else 0, part,
                counter, act.data_ptr() if act is not None else 0,
                iters.data_ptr() if (iters is not None and tol is not None) else 0,
                act.data_ptr() if act is not None else 0, 0,
                float(xsum if xsum is not None else 0.0), _stream_ptr(HT3))


def kl_sparse_loss(csr: KLCSR, HT3: torch.Tensor, W3: torch.Tensor, eps: float,
                   active: torch.Tensor | None = None,
                   st: torch.Tensor | None = None) -> torch.Tensor:
    """sum D_KL(X || HT3^T W3) per replicate over the CSR rows ``csr``, float64 (R,)."""
    R, K, N = HT3.shape
    _require_native()
    st = _sk_args(csr, HT3, W3, st)
    wsum = W3.sum(dim=2, dtype=torch.float32).contiguous()
    loss = torch.zeros((R, int(_hip.sk_groups(N, R, W3.shape[2], K))), dtype=torch.float64,
                       device=HT3.device)
    _hip.sk_run(0, csr.rowptr.data_ptr(), csr.col.data_ptr(), csr.val.data_ptr(), st.data_ptr(),
                st.stride(0), HT3.data_ptr(), HT3.stride(0), HT3.stride(1), K, N, W3.shape[2], R,
                float(eps),
                0, 0, 0, 1, wsum.data_ptr(), 0.0, 0.0, 0.0, 0, 0, 0, 0, 0, 0,
                active.data_ptr() if active is not None else 0, loss.data_ptr(), 0.0,
                _stream_ptr(HT3))
    lo, hi = int(csr.rowptr[0]), int(csr.rowptr[-1])
    return loss.sum(1) - csr.val[lo:hi].sum(dtype=torch.float64)


def kl_sparse_w_num(tiles: list, HT3: torch.Tensor, W3: torch.Tensor, eps: float,
                    active: torch.Tensor | None = None,
                    st: torch.Tensor | None = None) -> torch.Tensor:
    """KL spectra numerators num = HT Q over a row chunk given as :func:`kl_csr_tiles`
    (cells tiled so that each tile's usages fit in LDS), as (tiles, R, K, G) partials -- the
    :func:`beta_w_partials` layout (sparse_kl.hip side 1).  ``st``: :func:`kl_st` of HT3."""
    R, K, c = HT3.shape
    G = W3.shape[2]
    _require_native()
    if st is None:
        st = kl_st(HT3)
    if active is not None and (active.dtype != torch.int32 or active.numel() < R):
        raise ValueError("active: contiguous int32 with >= R entries")
    num = torch.empty((len(tiles), R, K, G), dtype=torch.float32, device=W3.device)
    for i, (t0, csrT) in enumerate(tiles):
        t1 = t0 + csrT.n_cols
        _sk_args(csrT, W3, HT3[:, :, t0:t1], st[:, t0:t1])
        sub = st[:, t0:t1]
        _hip.sk_run(1, csrT.rowptr.data_ptr(), csrT.col.data_ptr(), csrT.val.data_ptr(),
                    sub.data_ptr(), sub.stride(0), W3.data_ptr(), W3.stride(0), W3.stride(1), K,
                    G, t1 - t0, R, float(eps), num[i].data_ptr(), 1, 0, 0, 0, 0.0, 0.0, 0.0, 0,
                    0, 0, 0, 0, 0, active.data_ptr() if active is not None else 0, 0, 0.0,
                    _stream_ptr(W3))
    return num


# ----------------------------------------------------------------------------- gram
def gram(X3: torch.Tensor, out: torch.Tensor | None = None, accumulate: bool = False,
         active: torch.Tensor | None = None) -> torch.Tensor:
    """out[r] (+)= X3[r] X3[r]^T for X3 (R, K, n) with unit column stride (any row and
    replicate strides).  K <= 128: one MFMA workgroup per replicate (four for K > 64, one
    per 64 x 64 block; gram.hip); larger K: the library batched GEMM.  Replicates
    whose ``active`` flag is 0 keep their ``out`` untouched."""
    R, K, n = X3.shape
    if out is None:
        if accumulate:
            raise ValueError("accumulate needs an out tensor")
        out = torch.empty((R, K, K), device=X3.device, dtype=X3.dtype)
    native = use_native(X3)
    if native:
        _native_dtype_k("gram", X3.dtype, K, 1 << 30)
    if not native or K > 128:
        # (K > 128 on the GPU: a plain batched GEMM for the library, the rank-general
        # solve's system matrix -- solve_any.hip)
        g = torch.bmm(X3, X3.transpose(1, 2))
        if active is not None:
            keep = (active[:R] != 0).view(R, 1, 1)
            g = torch.where(keep, out + g if accumulate else g, out)
            out.copy_(g)
        elif accumulate:
            out += g
        else:
            out.copy_(g)
        return out
    if out.shape != (R, K, K) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("out must be a contiguous float32 (R, K, K) tensor")
    if n > 1 and X3.stride(2) != 1:
        raise ValueError("X3 needs unit column stride")
    if active is not None and (active.dtype != torch.int32 or active.numel() < R):
        raise ValueError("active: int32 with >= R entries")
    # few replicates: split the columns over S workgroups per replicate (one workgroup per
    # replicate left most of the chip idle at R = 8) and reduce the partials in order
    S = 1 if R >= _GRAM_SPLIT_MIN_R else max(1, min((n + 255) // 256, 512 // max(1, R)))
    part = 0
    if S > 1:
        ws = scratch(_GRAM_WS, (str(X3.device), _stream_ptr(X3)), S * R * K * K,
                     torch.float32, X3.device, 1 << 14)
        part = ws.data_ptr()
    _hip.gram(X3.data_ptr(), X3.stride(0), X3.stride(1), R, K, n, out.data_ptr(), K * K,
              int(bool(accumulate)), active.data_ptr() if active is not None else 0,
              part, int(S), _stream_ptr(X3))
    return out


_GRAM_WS: dict = {}

# scratch buffers a captured HIP graph has used: never freed while the process runs (a
# replaced cache entry would otherwise return memory a graph still writes to)
_GRAPH_HELD: list = []


def scratch(cache: dict, key, numel: int, dtype, device, min_numel: int = 0) -> torch.Tensor:
    """A per-key scratch tensor of >= ``numel`` elements from ``cache``, grown on demand.
    An entry handed out during a graph capture is marked; when a marked entry is replaced
    by a larger one, the old buffer is held for the life of the process (graphs captured
    with it keep its address)."""
    ent = cache.get(key)
    if ent is None or ent[0].numel() < numel:
        if ent is not None and ent[1]:
            _GRAPH_HELD.append(ent[0])
        ent = [torch.empty(max(numel, min_numel), dtype=dtype, device=device), False]
        cache[key] = ent
    if device.type == "cuda" and torch.cuda.is_current_stream_capturing():
        ent[1] = True
    return ent[0]
# replicate count from which one workgroup per replicate fills the chip (no column split)
_GRAM_SPLIT_MIN_R = 64
_gram_op = gram    # ops.solve's `gram` argument shadows the function there


# ----------------------------------------------------------------------------- consensus
def _f64_rows(t: torch.Tensor) -> torch.Tensor:
    t = t.to(torch.float64)
    return t if t.stride(-1) == 1 else t.contiguous()


def pairwise_dist(A: torch.Tensor, B: torch.Tensor | None = None,
                  squared: bool = False) -> torch.Tensor:
    """Euclidean distances between the rows of A (n, d) and B (m, d) in float64
    (sklearn euclidean_distances: |a|^2 + |b|^2 - 2ab clipped at 0, zero diagonal when B
    is A).  GPU: f64 MFMA tiles in consensus.hip."""
    same = B is None
    Ad = _f64_rows(A)
    Bd = Ad if same else _f64_rows(B)
    if Ad.shape[1] != Bd.shape[1]:
        raise ValueError("pairwise_dist: feature dimensions differ")
    na = (Ad * Ad).sum(dim=1)
    nb = na if same else (Bd * Bd).sum(dim=1)
    if not use_native(Ad):
        d2 = na[:, None] + nb[None, :] - 2.0 * (Ad @ Bd.t())
        d2.clamp_(min=0.0)
        if same:
            d2.fill_diagonal_(0.0)
        return d2 if squared else torch.sqrt(d2)
    n, m = Ad.shape[0], Bd.shape[0]
    D = torch.empty((n, m), dtype=torch.float64, device=Ad.device)
    _hip.pairdist(Ad.data_ptr(), Ad.stride(0), Bd.data_ptr(), Bd.stride(0), na.data_ptr(),
                  nb.data_ptr(), n, m, Ad.shape[1], D.data_ptr(), m, int(same), int(squared),
                  _stream_ptr(Ad))
    return D


def knn_sum(D: torch.Tensor, k: int) -> torch.Tensor:
    """Per row of the non-negative float64 matrix D, the sum of its k smallest entries
    (exact, ties included).  GPU: radix select in consensus.hip."""
    n, m = D.shape
    if not 1 <= k <= m:
        raise ValueError(f"knn_sum: need 1 <= k <= {m}, got {k}")
    if not use_native(D):
        return torch.topk(D, k, dim=1, largest=False).values.sum(dim=1)
    Dd = _f64_rows(D)
    out = torch.empty(n, dtype=torch.float64, device=D.device)
    _hip.knn_sum(Dd.data_ptr(), Dd.stride(0), n, m, int(k), out.data_ptr(), _stream_ptr(Dd))
    return out


def seg_argmin(D: torch.Tensor, k: int, row_add: torch.Tensor | None = None,
               col_add: torch.Tensor | None = None):
    """For D (n, nseg*k): per row and segment s, argmin_j (row_add[i] + col_add[s*k+j] +
    D[i, s*k+j]) and its value clipped at 0 -> (labels int64 (n, nseg), min float64)."""
    n, mm = D.shape
    if k < 1 or mm % k:
        raise ValueError("seg_argmin: columns must be a multiple of k")
    nseg = mm // k
    if not use_native(D):
        V = D.to(torch.float64)
        if row_add is not None:
            V = V + row_add.to(torch.float64)[:, None]
        if col_add is not None:
            V = V + col_add.to(torch.float64)[None, :]
        V = V.view(n, nseg, k)
        mn, lab = V.min(dim=2)
        return lab, mn.clamp(min=0.0)
    Dd = _f64_rows(D)
    ra = row_add.to(torch.float64).contiguous() if row_add is not None else None
    ca = col_add.to(torch.float64).contiguous() if col_add is not None else None
    lab = torch.empty((n, nseg), dtype=torch.int32, device=D.device)
    mind = torch.empty((n, nseg), dtype=torch.float64, device=D.device)
    _hip.seg_argmin(Dd.data_ptr(), Dd.stride(0), n, nseg, k, ra.data_ptr() if ra is not None else 0,
                    ca.data_ptr() if ca is not None else 0, lab.data_ptr(), mind.data_ptr(),
                    _stream_ptr(Dd))
    return lab.long(), mind


def small_gram(A: torch.Tensor, rows_are_points: bool = True) -> torch.Tensor:
    """K x K Gram of a tall operand on the device (segsum.hip small_gram_kernel; float32 /
    float64 as A): A^T A for A (n x K) (``rows_are_points``), else A A^T for A (K x n) --
    the consensus / refit / OLS Grams, without a library GEMM.  Row chunks summed in chunk
    order (deterministic)."""
    if A.dim() != 2:
        raise ValueError("small_gram: a 2-D operand")
    if rows_are_points:
        n, K = A.shape
        s_i, s_a = A.stride(0), A.stride(1)
    else:
        K, n = A.shape
        s_i, s_a = A.stride(1), A.stride(0)
    if not use_native(A) or K > 64 or A.dtype not in (torch.float32, torch.float64) or n == 0:
        return A.t() @ A if rows_are_points else A @ A.t()
    rows_per = max(64, -(-n // 256))
    chunks = -(-n // rows_per)
    part = torch.empty((chunks, K, K), dtype=A.dtype, device=A.device)
    _hip.small_gram(A.data_ptr(), s_i, s_a, n, K, A.element_size(), rows_per, part.data_ptr(),
                    _stream_ptr(A))
    return part.sum(0)


def seg_colsum(X: torch.Tensor, lab: torch.Tensor, k: int) -> torch.Tensor:
    """k-means centroid sums of every restart (segsum.hip, H4): for X (n, d) and labels
    ``lab`` (n_init, n) in [0, k), out[r, c] = sum of the rows i with lab[r, i] == c --
    float64, summed in point order (no one-hot matrix, no library GEMM)."""
    n, d = X.shape
    nr = lab.shape[0]
    if lab.dim() != 2 or lab.shape[1] != n or k < 1:
        raise ValueError(f"seg_colsum: lab (n_init, {n}) and k >= 1 required")
    if not use_native(X) or k > 256:     # (k > 256: the LDS tables do not fit; torch op)
        out = torch.zeros((nr, k, d), dtype=torch.float64, device=X.device)
        Xd = X.to(torch.float64)
        for r in range(nr):
            out[r].index_add_(0, lab[r].long(), Xd)
        return out
    Xd = _f64_rows(X)
    lb = lab.to(torch.int32).contiguous()
    out = torch.empty((nr, k, d), dtype=torch.float64, device=X.device)
    _hip.seg_colsum(Xd.data_ptr(), Xd.stride(0), n, d, lb.data_ptr(), lb.stride(0), nr, int(k),
                    out.data_ptr(), _stream_ptr(Xd))
    return out


def seg_rowsum(D: torch.Tensor, lab: torch.Tensor, k: int) -> torch.Tensor:
    """Per-row cluster sums of a distance matrix (segsum.hip, H6): for D (n, m) and column
    labels ``lab`` (m,) in [0, k), out[i, c] = sum_j D[i, j] over lab[j] == c -- float64
    in a fixed order (the silhouette's a / b terms, no one-hot GEMM)."""
    n, m = D.shape
    if lab.dim() != 1 or lab.shape[0] != m or k < 1:
        raise ValueError(f"seg_rowsum: lab ({m},) and k >= 1 required")
    if not use_native(D) or k > 256:
        out = torch.zeros((k, n), dtype=torch.float64, device=D.device)
        out.index_add_(0, lab.long(), D.to(torch.float64).t())
        return out.t().contiguous()
    Dd = _f64_rows(D)
    lb = lab.to(torch.int32).contiguous()
    out = torch.empty((n, k), dtype=torch.float64, device=D.device)
    _hip.seg_rowsum(Dd.data_ptr(), Dd.stride(0), n, m, lb.data_ptr(), int(k), out.data_ptr(),
                    out.stride(0), _stream_ptr(Dd))
    return out


def seg_median(S: torch.Tensor, rank: np.ndarray, k: int) -> torch.Tensor | None:
    """(k, G) per-cluster column medians of the float64 matrix S (n, G) for cluster ids
    ``rank`` (n,) in 0..k-1, every cluster non-empty (seg_median.hip: LDS rank counting,
    one workgroup per column, pandas' median of the two middle values).  None when the
    kernel's limits (n <= 4096 rows, k <= 256) do not hold -- the caller sorts instead."""
    n, G = S.shape
    if not use_native(S):
        return None
    if S.dtype != torch.float64 or (G > 1 and S.stride(1) != 1):
        raise ValueError("seg_median: float64 with unit column stride")
    if n > _hip.seg_median_max_rows() or k > _hip.seg_median_max_clusters():
        return None
    rank = np.asarray(rank, dtype=np.int64)
    counts = np.bincount(rank, minlength=k)
    if counts.size != k or (counts == 0).any():
        raise ValueError("seg_median: every cluster needs a member")
    perm = np.argsort(rank, kind="stable").astype(np.int32)
    seg = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    dev = S.device
    perm_t = torch.from_numpy(perm).to(dev)
    seg_t = torch.from_numpy(seg).to(dev)
    out = torch.empty((k, G), dtype=torch.float64, device=dev)
    _hip.seg_median(S.data_ptr(), S.stride(0), n, G, perm_t.data_ptr(), seg_t.data_ptr(), k,
                    out.data_ptr(), out.stride(0), _stream_ptr(S))
    return out


def kmeanspp_fused_ok(X: torch.Tensor, M: int) -> bool:
    """True when the fused k-means++ step (kmeans.hip kmeanspp_kernel) handles X (n, d) with
    M = n_init * trials candidates in LDS."""
    return use_native(X) and bool(_hip.kmeanspp_fits(int(M), int(X.shape[1])))


def kmeanspp_step(X: torch.Tensor, C: torch.Tensor, closest: torch.Tensor, trials: int,
                  update: bool = False):
    """Greedy k-means++ step for every restart (n_init = closest.shape[1]) without the
    (n x n_init*trials) distance matrix.  X (n, d) float64; C (n_init*trials, d) the
    candidates, restart r owning rows [r*trials, (r+1)*trials); closest (n, n_init) float64
    contiguous.  update=False: returns the potentials sum_i min(closest[i, r],
    |x_i - c_m|^2) as (n_init, trials); update=True (trials == 1): closest[i, r] =
    min(closest[i, r], |x_i - c_r|^2) in place.  GPU: kmeans.hip kmeanspp_kernel."""
    n, d = X.shape
    M = C.shape[0]
    n_init = closest.shape[1]
    if M != n_init * trials or closest.shape[0] != n or C.shape[1] != d:
        raise ValueError("kmeanspp_step: inconsistent shapes")
    if not use_native(X):
        D = ((X[:, None, :] - C[None, :, :]) ** 2).sum(dim=2).view(n, n_init, trials)
        V = torch.minimum(closest[:, :, None], D)
        if update:
            closest.copy_(V[:, :, 0])
            return None
        return V.sum(dim=0)
    Xd = _f64_rows(X)
    Cd = C.to(torch.float64).contiguous()
    if closest.dtype != torch.float64 or not closest.is_contiguous():
        raise ValueError("closest: contiguous float64 required")
    if not _hip.kmeanspp_fits(int(M), int(d)):
        raise ValueError(f"kmeanspp_step: M={M}, d={d} exceeds the fused kernel's LDS budget")
    if update:
        if trials != 1:
            raise ValueError("update needs one candidate per restart")
        _hip.kmeanspp(Xd.data_ptr(), Xd.stride(0), n, d, Cd.data_ptr(), M, 1,
                      closest.data_ptr(), n_init, 1, 0, _stream_ptr(X))
        return None
    nb = int(_hip.kmeanspp_blocks(n))
    pot = torch.empty((nb, M), dtype=torch.float64, device=X.device)
    _hip.kmeanspp(Xd.data_ptr(), Xd.stride(0), n, d, Cd.data_ptr(), M, trials,
                  closest.data_ptr(), n_init, 0, pot.data_ptr(), _stream_ptr(X))
    return pot.sum(dim=0).view(n_init, trials)


def kmeanspp_sample(closest: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    """k-means++ candidate draw for every restart: closest (n, n_init) float64 contiguous,
    u (n_init, trials) uniforms -> (n_init, trials) int64 point indices, the first point
    whose inclusive running sum of closest[:, r] reaches u * total (torch.searchsorted of
    the cumsum, clamped to n - 1).  GPU: kmeans.hip ppsum/ppsample kernels."""
    n, n_init = closest.shape
    if not use_native(closest) or _hip.kmeanspp_sample_blocks(n) > 15360:
        cum = torch.cumsum(closest.t().contiguous().double(), 1)
        return torch.searchsorted(cum, u * cum[:, -1:]).clamp(max=n - 1)
    if closest.dtype != torch.float64 or not closest.is_contiguous():
        raise ValueError("closest: contiguous float64 required")
    trials = u.shape[1]
    uu = u.to(torch.float64).contiguous()
    if uu.shape[0] != n_init:
        raise ValueError("u: one row per restart")
    nb = int(_hip.kmeanspp_sample_blocks(n))
    bsum = torch.empty((n_init, nb), dtype=torch.float64, device=closest.device)
    cand = torch.empty((n_init, trials), dtype=torch.int64, device=closest.device)
    _hip.kmeanspp_sample(closest.data_ptr(), n, n_init, uu.data_ptr(), trials, bsum.data_ptr(),
                         cand.data_ptr(), _stream_ptr(closest))
    return cand


def kmeans_fused_ok(X: torch.Tensor, k: int) -> bool:
    """True when the fused low-dimensional Lloyd step (kmeans.hip) handles (X, k)."""
    return use_native(X) and bool(_hip.kmeans_fits(int(k), int(X.shape[1])))


def kmeans_step(X: torch.Tensor, C: torch.Tensor, live: torch.Tensor | None = None,
                want_sums: bool = True, want_dist: bool = False):
    """One Lloyd step for every restart: X (n, d) float64, C (n_init, k, d) float64.

    Returns (labels int64 (n_init, n), sums (n_init, k, d) | None, counts (n_init, k) | None,
    mind float64 (n_init, n) | None): the nearest centroid of every point (exact squared
    distance, first index on ties), the per-cluster sums/counts of the assigned points
    (fixed-order, deterministic) and the squared distances.  Restarts with live == 0 are
    skipped on the GPU (their outputs are unspecified).  GPU: kmeans.hip."""
    n, d = X.shape
    n_init, k, d2 = C.shape
    if d2 != d:
        raise ValueError("kmeans_step: feature dimensions differ")
    Xd = _f64_rows(X)
    Cd = C.to(torch.float64).contiguous()
    if not use_native(Xd):
        xsq = (Xd * Xd).sum(dim=1)
        csq = (Cd * Cd).sum(dim=2)
        D = (xsq[None, :, None] + csq[:, None, :]
             - 2.0 * torch.einsum("nd,rkd->rnk", Xd, Cd)).clamp_(min=0.0)
        mind, lab = D.min(dim=2)
        sums = cnt = None
        if want_sums:
            sums = torch.zeros((n_init, k, d), dtype=torch.float64)
            cnt = torch.zeros((n_init, k), dtype=torch.float64)
            for r in range(n_init):
                sums[r].index_add_(0, lab[r], Xd)
                cnt[r].index_add_(0, lab[r], torch.ones(n, dtype=torch.float64))
        return lab, sums, cnt, (mind if want_dist else None)
    if not _hip.kmeans_fits(int(k), int(d)):
        raise ValueError(f"kmeans_step: k={k}, d={d} exceeds the fused kernel's LDS budget")
    dev = Xd.device
    nblk = int(_hip.kmeans_blocks(n))
    lab = torch.empty((n_init, n), dtype=torch.int32, device=dev)
    mind = torch.empty((n_init, n), dtype=torch.float64, device=dev) if want_dist else None
    psum = pcnt = None
    if want_sums:
        psum = torch.empty((nblk, n_init, k, d), dtype=torch.float64, device=dev)
        pcnt = torch.empty((nblk, n_init, k), dtype=torch.float64, device=dev)
    lv = live.to(device=dev, dtype=torch.int32).contiguous() if live is not None else None
    _hip.kmeans_step(Xd.data_ptr(), Xd.stride(0), n, d, Cd.data_ptr(), int(k), int(n_init),
                     lv.data_ptr() if lv is not None else 0, lab.data_ptr(),
                     mind.data_ptr() if mind is not None else 0,
                     psum.data_ptr() if psum is not None else 0,
                     pcnt.data_ptr() if pcnt is not None else 0, _stream_ptr(Xd))
    sums = psum.sum(dim=0) if want_sums else None
    cnt = pcnt.sum(dim=0) if want_sums else None
    return lab.long(), sums, cnt, mind


# ----------------------------------------------------------------------------- harmony
def harmony_native_ok(t: torch.Tensor, K: int, B: int) -> bool:
    """True when the fused Harmony R-update kernels handle this problem on ``t``'s device."""
    return use_native(t) and K <= 128 and K * B <= _hip.harmony_max_kb()


def harmony_block_update(Rt: torch.Tensor, distT: torch.Tensor | None, sigma: torch.Tensor,
                         cells: torch.Tensor, bidx: torch.Tensor, E: torch.Tensor,
                         O: torch.Tensor, Pr_b: torch.Tensor, theta: torch.Tensor,
                         ws: dict, Y: torch.Tensor | None = None, Zt: torch.Tensor | None = None,
                         obj: torch.Tensor | None = None, steps=(0, 1)) -> None:
    """One Harmony block update on device (harmony.hip): remove the block's old R from
    E/O and recompute the diversity penalty (step 0), reassign R for the block's cells and
    add it back (step 1).  Rt (N, K) float64 contiguous; cells int32 (nb,); bidx int32
    (nvar, N); E/O (K, B) float64.  ``distT`` (N, K) float64, or None: the distances
    2 (1 - Y_k . z_n) are formed inside the assign from ``Y`` (d, K) and ``Zt`` (N, d),
    and the assignment's objective terms (sum R dist, sum sigma R log R) are added to
    ``obj`` (2,) float64.  ``ws`` caches the partial-sum workspace and the penalty table
    (ws["pen"], which step 1 reads)."""
    N, K = Rt.shape
    B = E.shape[1]
    nvar = bidx.shape[0]
    nb = int(cells.numel())
    for name, t, dt in (("Rt", Rt, torch.float64), ("E", E, torch.float64),
                        ("O", O, torch.float64), ("cells", cells, torch.int32),
                        ("bidx", bidx, torch.int32)):
        if t.dtype != dt or not t.is_contiguous() or t.device != Rt.device:
            raise ValueError(f"{name}: contiguous {dt} on {Rt.device} required")
    if O.shape != (K, B) or bidx.shape[1] != N:
        raise ValueError("harmony_block_update: inconsistent shapes")
    d = 0
    if distT is None:
        if Y is None or Zt is None or obj is None:
            raise ValueError("harmony_block_update: Y, Zt and obj for the fused distances")
        d = int(Y.shape[0])
        for name, t, shp in (("Y", Y, (d, K)), ("Zt", Zt, (N, d)), ("obj", obj, (2,))):
            if t.dtype != torch.float64 or not t.is_contiguous() or tuple(t.shape) != shp:
                raise ValueError(f"{name}: contiguous float64 {shp} required")
    elif distT.dtype != torch.float64 or not distT.is_contiguous() or distT.shape != (N, K):
        raise ValueError("distT: contiguous float64 (N, K) required")
    # ~512 workgroups of up to 4 waves (2 per CU): each wave walks a few dozen cells
    chunk = max(16, -(-nb // 512))
    n_wg = -(-nb // chunk)
    need = n_wg * (K * (B + 1) + 2)
    if ws.get("part") is None or ws["part"].numel() < need:
        ws["part"] = torch.empty(need, dtype=torch.float64, device=Rt.device)
    if ws.get("pen") is None:
        ws["pen"] = torch.empty((K, B), dtype=torch.float64, device=Rt.device)
    st = _stream_ptr(Rt)
    args = (Rt.data_ptr(), distT.data_ptr() if distT is not None else 0, sigma.data_ptr(),
            cells.data_ptr(), bidx.data_ptr(), nb, N, K, B, nvar, chunk, E.data_ptr(),
            O.data_ptr(), Pr_b.data_ptr(), theta.data_ptr(), ws["pen"].data_ptr(),
            ws["part"].data_ptr(), Y.data_ptr() if Y is not None else 0,
            Zt.data_ptr() if Zt is not None else 0, d, obj.data_ptr() if obj is not None else 0,
            st)
    for op in steps:
        _hip.harmony_block(op, *args)


def harmony_centroids_ok(d: int, K: int) -> bool:
    """True when the centroid kernel (and the fused-distance assign) take d PCs x K
    clusters: one lane per PC, 4 x 8 MFMA tiles."""
    return 1 <= d <= int(_hip.harmony_centroid_max_d()) and 1 <= K <= 128


def harmony_centroids(Zt: torch.Tensor, Rt: torch.Tensor, ws: dict) -> torch.Tensor:
    """Y = Z_cos R^T (d, K) from the cell-major Zt (N, d) and Rt (N, K), float64, on the
    device in two deterministic stages (harmony.hip: chunked partials, per-output wave
    sums) -- never a library GEMM with one output tile walking every cell."""
    N, d = Zt.shape
    K = Rt.shape[1]
    for name, t in (("Zt", Zt), ("Rt", Rt)):
        if t.dtype != torch.float64 or not t.is_contiguous() or t.shape[0] != N:
            raise ValueError(f"harmony_centroids: {name} contiguous float64 with N rows")
    if not harmony_centroids_ok(d, K):
        raise ValueError(f"harmony_centroids: d = {d}, K = {K} beyond the kernel's tiles")
    # ~1024 workgroups (4 per CU), whole 4-cell MFMA steps
    chunk = max(64, -(-N // 1024))
    chunk = -(-chunk // 4) * 4
    n_wg = -(-N // chunk)
    need = n_wg * d * K
    if ws.get("cpart") is None or ws["cpart"].numel() < need:
        ws["cpart"] = torch.empty(need, dtype=torch.float64, device=Zt.device)
    Y = torch.empty((d, K), dtype=torch.float64, device=Zt.device)
    _hip.harmony_centroid(Zt.data_ptr(), Rt.data_ptr(), N, d, K, chunk, ws["cpart"].data_ptr(),
                          Y.data_ptr(), _stream_ptr(Zt))
    return Y


def harmony_objective(O: torch.Tensor, E: torch.Tensor, sigma: torch.Tensor,
                      theta: torch.Tensor, obj: torch.Tensor, out: torch.Tensor) -> None:
    """out[0] = obj[0] + obj[1] + sum_{k,b} sigma_k theta_b O log((O + 1) / (E + 1)) (the
    round's Harmony objective from the assign passes' sums and the cross-entropy term,
    which O = R Phi^T reduces to K x B numbers); resets obj."""
    K, B = O.shape
    _hip.harmony_objective(O.data_ptr(), E.data_ptr(), sigma.data_ptr(), theta.data_ptr(), K, B,
                           obj.data_ptr(), out.data_ptr(), _stream_ptr(O))


# ----------------------------------------------------------------------------- init
def philox_fill(out: torch.Tensor, seeds: torch.Tensor, scales: torch.Tensor, stream: int,
                mode: int = 0, row_offset: int = 0) -> None:
    """Fill ``out`` viewed as (R, rows, cols) (any strides) with replicate r's Philox
    stream: ``|N(0,1)|*scale[r]`` (mode 0) or ``U(0,1)*scale[r]`` (mode 1)."""
    if out.dim() != 3:
        raise ValueError("out must be (R, rows, cols)")
    R, rows, cols = out.shape
    if seeds.numel() != R or scales.numel() != R:
        raise ValueError("one seed and one scale per replicate")
    if not use_native(out) or out.dtype != torch.float32:
        return reference.philox_fill(out, seeds, scales, stream, mode, row_offset)
    seeds_d = seeds.to(device=out.device, dtype=torch.int64).contiguous()
    scales_d = scales.to(device=out.device, dtype=torch.float32).contiguous()
    _hip.philox_fill(out.data_ptr(), rows, cols, out.stride(1), out.stride(2), out.stride(0),
                     int(row_offset), seeds_d.data_ptr(), scales_d.data_ptr(), R, int(stream),
                     int(mode), _stream_ptr(out))


# ----------------------------------------------------------------------------- split GEMM
def planes_bk(pb: int) -> int:
    """k granularity the split-precision GEMM's plane buffers are padded to (a multiple of
    both k-step depths, 32 and 64)."""
    return 64


def gemm_kstep(variant: int) -> int:
    """k-step depth (BK) of the split GEMM: 64 = two MFMA k-steps per LDS stage and barrier
    (the kernel drops to 32 where a 64-deep stage pair would not fit in LDS, or Kd is not
    a multiple of 64).  Measured on MI355X (profiles/r2_gemm_bk_sweep.txt): the 8-wave
    128x256 tiles gain (K=10 statistics GEMM 62 -> 60 us, K-grid GEMMs 410/393 -> 400/381 us,
    as 2 stages of 64 against 3 of 32), the 2- and 4-wave tiles lose (64x128 numerator
    77 -> 97 us).  CNMF_GEMM_BK overrides (A/B runs)."""
    if _ENV["CNMF_GEMM_BK"]:
        return int(_ENV["CNMF_GEMM_BK"])
    return 64 if variant in (1, 2, 5) else 32


_GEMM_TILES = {0: (128, 128), 1: (128, 256), 2: (256, 128), 3: (64, 128), 4: (64, 128),
               5: (128, 128)}
_GEMM_SLAB: dict = {}


def gemm_a_planes(Kd: int) -> int:
    """A planes the engine's split GEMMs use for a reduction of length Kd: 2 (hi + mid,
    representation error <= 2^-16 relative) once Kd >= 1024 -- that bound is inside the
    fp32 GEMM's own n * 2^-24 bound from n = 256 on, and from ~1000 on the measured error
    is also below the fp32 library GEMM's (test_gemm_two_a_planes_within_fp32_library_error)
    -- else 3 (exact)."""
    return 3 if Kd < 1024 else 2


def gemm_plan(M: int, N: int, Kd: int, pb: int) -> tuple[int, int]:
    """(tile variant, k split) for an M x N x Kd split GEMM: the largest tile that still
    gives every CU a workgroup, else k-split slices (deterministic slab reduction) until
    ~2 workgroups per CU.  CNMF_GEMM_VARIANT / CNMF_GEMM_KSPLIT override (benchmarks)."""
    cus = 256
    nk = Kd // planes_bk(pb)
    v_env, k_env = _ENV["CNMF_GEMM_VARIANT"], _ENV["CNMF_GEMM_KSPLIT"]

    def tiles(v):
        tm, tn = _GEMM_TILES[v]
        return -(-M // tm) * -(-N // tn)

    # measured on MI355X (profiles/r2_gemm_planes_sweep.log): 128x256 tiles win once they
    # alone fill the chip; 64x128 tiles when those give two workgroups per CU without a
    # k split (no reduction pass); 128x256 with a k split for few, long tiles; and for a
    # few rows (the tail passes) 128x128 tiles with a deep k split
    target = cus
    if v_env is not None:
        v = int(v_env)
    elif tiles(1) >= cus:
        v = 1
    elif tiles(3) >= 2 * cus:
        # 64 x 128 tiles as 4 waves of 32 x 64 (variant 4): twice the waves per output to
        # hide LDS / barrier latency -- K=10 numerator 63.4 -> 60.1 us in the bench
        # (profiles/r2_gemm_small_tile_sweep.log; 2 waves of 64 x 64, variant 3, lost)
        v = 4
    elif M > 128:
        v = 1
    else:
        v, target = 0, 2 * cus
    ksplit = 1
    if k_env is not None:
        ksplit = int(k_env)
    elif v_env is None and 1024 < M <= 4096:
        # K x replicates in (1024, 4096] (K = 11..40 at 100 replicates): 128 x 256 tiles
        # with the k split that best fills whole waves of CUs -- cost ~ ceil(units / CUs)
        # / ksplit per unit of work + 0.13 per extra split (slab traffic).  Measured
        # (tools/gemm_plan_sweep.py, profiles/r4q_*): K=20 numerator 99.9 -> 86.7 us,
        # statistics 85.0 -> 65.9; K=30 statistics 128.4 -> 115.1; K=30 numerator kept.
        # Bench (profiles/r4r_*): K=20 5,325 -> 5,437, K=30 3,661 -> 3,738 rep/s; at K=50
        # (M = 5000) the extra slabs cost the solves more than the GEMMs gain (1,300 ->
        # 1,211), so larger M keeps the rule below
        t = tiles(1)
        best = None
        for ks in (1, 2, 4):
            if nk // ks < 4:
                break
            cost = -(-t * ks // cus) / ks + 0.13 * (ks - 1)
            if best is None or cost < best[0] - 1e-9:
                best = (cost, ks)
        return 1, best[1] if best else 1
    else:
        t = tiles(v)
        while t * ksplit < target and nk // (2 * ksplit) >= 4:
            ksplit *= 2
    return v, max(1, min(ksplit, nk))


def split_planes(S: torch.Tensor, out: torch.Tensor, col_mul: torch.Tensor | None = None) -> None:
    """Exact bf16 split of the fp32 matrix ``S`` (rows, cols; unit column stride), times
    the optional per-column factor ``col_mul``, into ``out`` (P, rows_out >= rows,
    cols_pad) int16 (bf16 bit patterns; any 4-aligned row pitch): plane 0 = rn(v),
    plane 1 = rn(v - plane 0), plane 2 = rn of the rest (v == sum of the planes for every
    normal fp32 value when P == 3).  Columns [cols, cols_pad) are written as zeros (the
    GEMM's k padding)."""
    rows, cols = S.shape
    P_, rows_out, ld = out.shape
    pitch = out.stride(1)
    if out.dtype != torch.int16 or out.stride(2) != 1 or rows_out < rows or pitch % 4 \
            or out.stride(0) % 4 or ld > pitch or out.data_ptr() % 8:
        raise ValueError("out: int16 (P, rows, cols_pad) planes, unit column stride, "
                         "4-aligned pitches, 8-byte aligned base")
    if cols > ld or ld % 4 or not 1 <= P_ <= 3:
        raise ValueError(f"split_planes: cols {cols} vs cols_pad {ld}, planes {P_}")
    if S.dtype != torch.float32 or (cols > 1 and S.stride(1) != 1):
        raise ValueError("S: float32 with unit column stride required")
    if col_mul is not None and (col_mul.dtype != torch.float32 or col_mul.numel() < cols
                                or not col_mul.is_contiguous()):
        raise ValueError("col_mul: contiguous float32 with >= cols entries")
    if not use_native(S):
        out[:, :rows].copy_(reference.split_planes(S if col_mul is None else S * col_mul[:cols],
                                                   P_, ld))
        return
    _hip.split_planes(S.data_ptr(), S.stride(0), rows, cols, ld,
                      col_mul.data_ptr() if col_mul is not None else 0, out.data_ptr(), pitch,
                      out.stride(0), P_, _stream_ptr(S))


def gemm_planes(C: torch.Tensor | None, A: torch.Tensor, B: torch.Tensor, M: int, N: int,
                Kd: int, accumulate: bool = False, col_scale: torch.Tensor | None = None,
                raw_slab: torch.Tensor | None = None, raw_max: int = 1 << 30,
                gate: torch.Tensor | None = None, plan: tuple | None = None) -> int:
    """C[:M, :N] (+)= col_scale * sum_{i + j <= 2} A[i][:M, :Kd] . B[j][:N, :Kd]^T on the bf16
    matrix cores (gemm_planes.hip): the fp32-accurate product of the fp32 matrices whose
    exact bf16 splits are A (3 planes; or its first 2, see gemm_a_planes) and B (1-3
    planes; 1 or 2 when B holds integers).
    A/B: int16 (P, rows, ld) views with unit k stride (row offsets / k offsets are just
    views); k must be zero-padded in A up to ``Kd`` (a multiple of 32; of planes_bk for
    the deep k-step).

    ``raw_slab`` (float32, >= ksplit * M * N elements; ``C`` unused, may be None): the raw
    split-K partial products go to ``raw_slab`` as [ksplit][M][N] WITHOUT the reduction
    pass, col_scale or accumulation -- the consuming solve sums them in slice order
    (ops.solve ``numer_slabs``), bitwise the same as the reduction.  When the plan splits
    k more than ``raw_max`` ways, the product is reduced here instead (into the first
    M x N floats of ``raw_slab``): a consumer reading that many slabs per element costs
    more than the reduction pass.  Returns the number of slabs in ``raw_slab`` (raw
    mode; 1 otherwise).  ``gate`` (int32 device scalar, GPU only): the kernels return at
    once when it holds 0 (conv_update's "no replicate active": the speculative pass
    after a batch finished)."""
    pa, a_rows, _ = A.shape
    pb, b_rows, _ = B.shape
    for name, t in (("A", A), ("B", B)):
        if t.dtype != torch.int16 or t.stride(2) != 1 or t.stride(1) % 8 or t.stride(0) % 8:
            raise ValueError(f"{name}: int16 planes with unit k stride, 8-aligned strides")
        if t.data_ptr() % 16:
            raise ValueError(f"{name}: 16-byte aligned base required (k offset % 8 == 0)")
        if t.shape[2] < Kd:
            raise ValueError(f"{name}: k extent {t.shape[2]} < Kd {Kd}")
    if not 2 <= pa <= 3 or not 1 <= pb <= 3 or Kd % 32 or M > a_rows or N > b_rows:
        raise ValueError(f"gemm_planes: planes {pa}/{pb}, Kd {Kd}, M {M}/{a_rows}, N {N}/{b_rows}")
    if raw_slab is not None:
        if raw_slab.dtype != torch.float32 or not raw_slab.is_contiguous():
            raise ValueError("raw_slab: contiguous float32 required")
        if C is None:
            C = raw_slab.view(-1)[:M * N].view(M, N)
    if C.dtype != torch.float32 or C.stride(1) != 1 or C.shape[0] < M or C.shape[1] < N:
        raise ValueError("C: float32 (>= M, >= N) with unit column stride required")
    if col_scale is not None and (col_scale.dtype != torch.float32 or col_scale.numel() < N
                                  or not col_scale.is_contiguous()):
        raise ValueError("col_scale: contiguous float32 with >= N entries")
    if not use_native(C):
        prod = reference.gemm_planes(A[:, :M, :Kd], B[:, :N, :Kd])
        if raw_slab is not None:
            raw_slab.view(-1)[:M * N].copy_(prod.to(torch.float32).reshape(-1))
            return 1
        if col_scale is not None:
            prod = prod * col_scale[:N].double()
        if accumulate:
            C[:M, :N] += prod.to(C.dtype)
        else:
            C[:M, :N] = prod.to(C.dtype)
        return
    variant, ksplit = plan if plan is not None else gemm_plan(M, N, Kd, pb)
    slab = 0
    if raw_slab is not None and ksplit > raw_max:
        # (capping ksplit at raw_max instead -- no reduction pass, fewer workgroups -- was
        # slower on the tail passes: 232 vs 212 us, profiles/r3s_*)
        gemm_planes(C, A, B, M, N, Kd, accumulate=False, col_scale=None, gate=gate)
        return 1
    if raw_slab is not None:
        if raw_slab.numel() < ksplit * M * N:
            raise ValueError(f"raw_slab: {raw_slab.numel()} < ksplit {ksplit} x {M} x {N}")
        slab = raw_slab.data_ptr()
    elif ksplit > 1:
        ws = scratch(_GEMM_SLAB, (str(C.device), _stream_ptr(C)), ksplit * M * N,
                     torch.float32, C.device, 1 << 20)
        slab = ws.data_ptr()
    _hip.gemm_planes(A.data_ptr(), A.stride(1), A.stride(0), a_rows, B.data_ptr(), B.stride(1),
                     B.stride(0), b_rows, C.data_ptr(), C.stride(0),
                     col_scale.data_ptr() if col_scale is not None else 0, int(M), int(N),
                     int(Kd), pa, pb, int(bool(accumulate)), int(variant), int(ksplit), slab,
                     gemm_stages(variant), gemm_kstep(variant), int(raw_slab is not None),
                     _gate_ptr(gate, C.device), _stream_ptr(C))
    return ksplit if raw_slab is not None else 1


def _gate_ptr(gate, dev) -> int:
    if gate is None:
        return 0
    if gate.dtype != torch.int32 or gate.numel() < 1 or gate.device != dev:
        raise ValueError("gate: int32 device tensor with >= 1 element")
    return gate.data_ptr()


def gemm_stages(variant: int) -> int:
    """LDS pipeline depth of the split GEMM (k-steps in flight + 1; the kernel drops to 2
    where 3 stages would not fit in LDS).  Measured on MI355X
    (profiles/r2_gemm_stages_sweep.txt): the 8-wave tiles (128x256, 256x128; one
    workgroup per CU) gain from a third stage (stats GEMM of the K-grid 442 -> 407 us),
    the 2- and 4-wave tiles lose more occupancy than they gain latency cover (64x128
    numerator 80 -> 108 us).  CNMF_GEMM_STAGES overrides (A/B runs)."""
    if _ENV["CNMF_GEMM_STAGES"]:
        return int(_ENV["CNMF_GEMM_STAGES"])
    return 3 if variant in (1, 2, 5) else 2


# ----------------------------------------------------------------------------- column stats
def colstats(X: torch.Tensor):
    """Per column of the fp32 matrix X (unit column stride): smallest positive entry
    (inf if none), float64 sum of squares, any-negative flag -- one pass, deterministic
    (colstats.hip)."""
    N, G = X.shape
    if X.dtype != torch.float32 or (G > 1 and X.stride(1) != 1):
        raise ValueError("colstats: float32 with unit column stride required")
    if not use_native(X):
        return reference.colstats(X)
    dev = X.device
    nb = int(_hip.colstats_blocks(N))
    pmin = torch.empty((nb, G), dtype=torch.float32, device=dev)
    psq = torch.empty((nb, G), dtype=torch.float64, device=dev)
    pneg = torch.empty((nb, G), dtype=torch.int32, device=dev)
    mn = torch.empty(G, dtype=torch.float32, device=dev)
    sq = torch.empty(G, dtype=torch.float64, device=dev)
    neg = torch.empty(G, dtype=torch.int32, device=dev)
    _hip.colstats(X.data_ptr(), X.stride(0), N, G, pmin.data_ptr(), psq.data_ptr(),
                  pneg.data_ptr(), mn.data_ptr(), sq.data_ptr(), neg.data_ptr(), _stream_ptr(X))
    return mn, sq, neg


def count_unit_check(X: torch.Tensor, mn: torch.Tensor) -> torch.Tensor:
    """int32 (G,) bit masks: bit d-1 set when some entry of the column is not an integer
    multiple of mn/d (d = 1..8) to fp32 rounding (or the multiple exceeds 65535)."""
    N, G = X.shape
    if not use_native(X):
        return reference.count_unit_check(X, mn)
    bad = torch.zeros(G, dtype=torch.int32, device=X.device)
    _hip.count_unit_check(X.data_ptr(), X.stride(0), N, G, mn.contiguous().data_ptr(),
                          bad.data_ptr(), _stream_ptr(X))
    return bad


# ----------------------------------------------------------------------------- H8
def predict_err_terms(X: torch.Tensor, U: torch.Tensor, S: torch.Tensor) -> tuple[float, float]:
    """(<X, U S>, ||X||^2) in float64 for a resident dense X (N x G, float32, unit column
    stride), usages U (N x K) and spectra S (K x G) -- the two data terms of the trace
    identity ||X - U S||^2 = ||X||^2 - 2 <X, U S> + <U^T U, S S^T> (cnmf.py:1100-1104).
    GPU: ONE pass over X (csrc/kernels/predict_err.hip: the U S tile on the f64 matrix
    cores, folded with X in registers; U S never materialised).  CPU: float64 torch."""
    N, G = X.shape
    K = U.shape[1]
    if U.shape[0] != N or S.shape != (K, G):
        raise ValueError(f"predict_err_terms: X {tuple(X.shape)}, U {tuple(U.shape)}, "
                         f"S {tuple(S.shape)}")
    if not use_native(X):
        Xd = X.to(torch.float64)
        return float((Xd * (U.to(torch.float64) @ S.to(torch.float64))).sum()), \
            float((Xd * Xd).sum())
    if X.dtype != torch.float32 or (G > 1 and X.stride(1) != 1):
        raise ValueError("X: float32 with unit column stride")
    if K > 128:
        raise ValueError(f"predict_err_terms: K={K} > 128")
    Ud = U.to(device=X.device, dtype=torch.float64).contiguous()
    Sd = S.to(device=X.device, dtype=torch.float64).contiguous()
    part = torch.empty(2 * (-(-N // 64)), dtype=torch.float64, device=X.device)
    _hip.predict_err(X.data_ptr(), X.stride(0), Ud.data_ptr(), K, Sd.data_ptr(), G, N, G, K,
                     part.data_ptr(), _stream_ptr(X))
    t = part.view(-1, 2).sum(dim=0).cpu()
    return float(t[0]), float(t[1])


# ----------------------------------------------------------------------------- exact stats
EXACT_D1, EXACT_D2 = 13, 25     # digits of sum x / sum x^2 (csrc/kernels/exact_moments.hip)


def exact_moments(X: torch.Tensor, acc: torch.Tensor | None = None,
                  bad_acc: torch.Tensor | None = None):
    """Exact per-column (sum x, sum x^2) of a dense device matrix (float32 / float64, unit
    column stride) as integer digits ((G, 13), (G, 25) int64 numpy) plus the count of
    values outside the exact window -- the same integers as the host path
    (models.hvg.exact_moment_digits), so statistics do not depend on the device or on how
    the rows are split (csrc/kernels/exact_moments.hip).  With ``acc`` ((G, 38) int64
    device) and ``bad_acc`` ((1,) int64 device) the digits are ADDED there instead (row
    blocks of a larger matrix; integer sums, exact) and nothing is returned."""
    if not use_native(X):
        raise ValueError("exact_moments: a device tensor is required")
    if X.dim() != 2 or X.dtype not in (torch.float32, torch.float64) or \
            (X.shape[1] > 1 and X.stride(1) != 1):
        raise ValueError("exact_moments: 2-D float32/float64 with unit column stride")
    rows, G = X.shape
    D = EXACT_D1 + EXACT_D2
    chunks = max(1, min(256, -(-rows // 4096), (1 << 14) // max(1, -(-G // 128))))
    part = torch.empty(chunks * G * D, dtype=torch.int64, device=X.device)
    out = torch.empty((G, D), dtype=torch.int64, device=X.device)
    bad = torch.zeros(1, dtype=torch.int64, device=X.device)
    _hip.exact_moments(X.data_ptr(), int(X.dtype == torch.float64), X.stride(0), rows, G, chunks,
                       part.data_ptr(), out.data_ptr(), bad.data_ptr(), _stream_ptr(X))
    if acc is not None:
        acc += out
        bad_acc += bad
        return None
    o = out.cpu().numpy()
    return o[:, :EXACT_D1].copy(), o[:, EXACT_D1:].copy(), int(bad.item())


# the rank-general paths (solve_any.hip, beta_any.hip): ranks beyond the tiled kernels
from .rank_general import (  # noqa: E402
    _beta_contract_any,
    _solve_any,
    beta_any_k,
    solve_any_k,
    solve_any_max_k,
)
