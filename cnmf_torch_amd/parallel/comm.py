"""Communicator abstraction used by the solvers.

``LocalComm`` is the single-process no-op.  ``DistComm`` wraps a ``torch.distributed``
process group: backend ``nccl`` (= RCCL on ROCm, over xGMI between the GPUs of a
node) for device tensors, ``gloo`` for CPU tests; ``CNMF_ALLREDUCE=xgmi`` routes device
all-reduce / reduce-scatter / all-gather calls to the one-shot peer-memory kernels
(parallel/xgmi.py).  Per online step the cell-sharded solvers issue ONE collective of
the flat ``[B | A]`` statistics (unfused step: all-reduce) or one packed reduce-scatter
and one packed all-gather (fused step), SURVEY.md §2.6 item 1, plus a few scalars at
init, so the interface is small.
"""
from __future__ import annotations

import torch


class _Done:
    """Handle of a collective that completed when it was issued."""
    __slots__ = ()

    def wait(self) -> None:
        return None


_DONE = _Done()


class _SideStreamWork:
    """Handle of a one-shot xGMI collective running on the communicator's side stream:
    wait() orders the CURRENT stream after it (no host sync)."""
    __slots__ = ("ev",)

    def __init__(self, ev):
        self.ev = ev

    def wait(self) -> None:
        torch.cuda.current_stream().wait_event(self.ev)


class LocalComm:
    rank = 0
    world_size = 1

    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        return t

    def allreduce_scalar(self, v: float) -> float:
        return float(v)

    def allreduce_max_int(self, v: int) -> int:
        return int(v)

    def barrier(self) -> None:
        pass

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        return t

    def all_gather_object(self, obj):
        return [obj]

    def gather_object(self, obj, dst: int = 0):
        return [obj]

    def send_object(self, obj, dst: int) -> None:
        raise RuntimeError("single process: nothing to send to")

    def recv_object(self, src: int):
        raise RuntimeError("single process: nothing to receive")

    def all_gather_(self, t: torch.Tensor) -> list[torch.Tensor]:
        return [t]

    def reduce_scatter_(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """out = this rank's chunk of the sum over ranks of ``inp`` (world equal chunks,
        contiguous, rank-major)."""
        out.copy_(inp.reshape(-1)[:out.numel()].view_as(out))
        return out

    def all_gather_into_(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """out (world equal chunks, rank-major, contiguous) = every rank's ``inp``."""
        out.reshape(-1)[:inp.numel()].copy_(inp.reshape(-1))
        return out

    # asynchronous forms (the DP fused step overlaps each exchange with the next unit's
    # compute, models/nmf_dp.py): issue now, ``.wait()`` on the returned handle orders
    # the current stream after the collective.  Here (and wherever a backend cannot run
    # one in the background) the collective completes when issued.
    def reduce_scatter_async(self, out: torch.Tensor, inp: torch.Tensor):
        self.reduce_scatter_(out, inp)
        return _DONE

    def all_gather_into_async(self, out: torch.Tensor, inp: torch.Tensor):
        self.all_gather_into_(out, inp)
        return _DONE

    @property
    def is_distributed(self) -> bool:
        return False


class DistComm(LocalComm):
    """torch.distributed-backed communicator (one process per GPU)."""

    def __init__(self, group=None):
        import torch.distributed as dist

        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised")
        self._dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self._xgmi = None           # one-shot xGMI all-reduce (CNMF_ALLREDUCE=xgmi), lazy
        self._side = None           # the stream every one-shot xGMI collective runs on
        # when a list: every device collective appends (kind, in numel, out numel, dtype)
        # -- bench.py --mode dp replays one step's sequence to time the collective term
        self.record = None

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    def _dev(self):
        if self.backend == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def _xgmi_for(self, t: torch.Tensor, any_dtype: bool = False):
        """The one-shot xGMI collectives when they are enabled and take ``t`` (float32
        device buffers up to its capacity -- any dtype for an all-gather, which moves bit
        patterns; parallel/xgmi.py), else None.  Created collectively on the first device
        collective: every rank of a DP solve issues the same sequence."""
        if t.device.type != "cuda":
            return None
        if self._xgmi is None:
            from . import xgmi

            self._xgmi = False
            if xgmi.wanted():
                try:
                    self._xgmi = xgmi.XgmiAllReduce(self.group, t.device)
                except xgmi.XgmiUnavailable as e:     # same decision on every rank
                    import warnings

                    warnings.warn(f"CNMF_ALLREDUCE=xgmi unavailable ({e}); using RCCL")
        if not self._xgmi:
            return None
        return self._xgmi if (any_dtype or self._xgmi.supports(t)) else None

    def _on_side(self, fn):
        """Run the one-shot xGMI launch ``fn`` on the side stream, after everything
        issued so far on the current stream; returns (fn's result, handle).  EVERY xGMI
        collective goes through here, so they keep one order on one stream (they share
        the device epoch and the peer staging) while compute proceeds beside them."""
        cur = torch.cuda.current_stream()
        if self._side is None:
            # the collectives' own stream: launches on it run without a further fork
            self._side = self._xgmi.stream if self._xgmi else torch.cuda.Stream(device=cur.device)
        self._side.wait_stream(cur)
        with torch.cuda.stream(self._side):
            ok = fn()
        ev = torch.cuda.Event()
        ev.record(self._side)
        return ok, _SideStreamWork(ev)

    def check(self) -> None:
        """Raise if a one-shot xGMI all-reduce gave up on a peer (host sync)."""
        if self._xgmi:
            self._xgmi.check()

    def close(self) -> None:
        if self._side is not None:
            self._side.synchronize()
        if self._xgmi:
            self._xgmi.close()
        self._xgmi = None

    def _rec(self, kind: str, inp: torch.Tensor, out: torch.Tensor) -> None:
        if getattr(self, "record", None) is not None and inp.is_cuda:
            self.record.append((kind, inp.numel(), out.numel(), inp.dtype))

    def replay(self, calls, reps: int = 10) -> float:
        """Seconds per replay of a recorded collective sequence (``record``), each call
        issued as in the solve and waited for on the current stream: the collective term
        of one step on this fabric, timed between barriers."""
        dev = torch.device("cuda", torch.cuda.current_device())
        bufs = [(k, torch.zeros(ni, dtype=dt, device=dev), torch.zeros(no, dtype=dt, device=dev))
                for k, ni, no, dt in calls]

        def once():
            for k, a, b in bufs:
                if k == "all_reduce":
                    self.allreduce_(a)
                elif k == "reduce_scatter":
                    self.reduce_scatter_(b, a)
                else:
                    self.all_gather_into_(b, a)

        once()
        self.barrier()
        torch.cuda.synchronize()
        import time as _t

        t0 = _t.perf_counter()
        for _ in range(reps):
            once()
        torch.cuda.synchronize()
        el = _t.perf_counter() - t0
        self.barrier()
        return el / max(1, reps)

    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.world_size == 1:
            return t
        self._rec("all_reduce", t, t)
        xg = self._xgmi_for(t)
        if xg is not None:
            self._on_side(lambda: xg(t))[1].wait()
            return t
        if (self.backend == "nccl") != (t.device.type == "cuda"):
            # stage through the backend's device: gloo reduces host tensors, RCCL device
            # ones (a host int64 digit vector from the sharded prepare's exact moments
            # travels over RCCL exactly -- integer sums are order-independent)
            st = t.to(self._dev(), copy=True)
            self._dist.all_reduce(st, group=self.group)
            t.copy_(st)
            return t
        self._dist.all_reduce(t, group=self.group)
        return t

    def allreduce_scalar(self, v: float) -> float:
        if self.world_size == 1:
            return float(v)
        t = torch.tensor([float(v)], dtype=torch.float64, device=self._dev())
        self._dist.all_reduce(t, group=self.group)
        return float(t.item())

    def allreduce_max_int(self, v: int) -> int:
        if self.world_size == 1:
            return int(v)
        t = torch.tensor([int(v)], dtype=torch.int64, device=self._dev())
        self._dist.all_reduce(t, op=self._dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def barrier(self) -> None:
        if self.world_size > 1:
            if self.backend == "nccl":
                self._dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
            else:
                self._dist.barrier(group=self.group)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.world_size > 1:
            self._dist.broadcast(t, src=src, group=self.group)
        return t

    def all_gather_object(self, obj):
        if self.world_size == 1:
            return [obj]
        out = [None] * self.world_size
        self._dist.all_gather_object(out, obj, group=self.group)
        return out

    def all_gather_(self, t: torch.Tensor) -> list[torch.Tensor]:
        """Every rank's ``t`` (same shape and dtype everywhere), in rank order.  Device
        tensors travel over RCCL (one ring all-gather on the xGMI links); under gloo a
        device tensor is staged through the host."""
        if self.world_size == 1:
            return [t]
        src = t if (self.backend == "nccl") == (t.device.type == "cuda") else \
            t.to(self._dev())
        out = [torch.empty_like(src) for _ in range(self.world_size)]
        self._dist.all_gather(out, src.contiguous(), group=self.group)
        return out if src is t else [o.to(t.device) for o in out]

    def reduce_scatter_(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """One reduce-scatter (RCCL ring on the xGMI links): ``out`` = chunk ``rank`` of
        the sum over ranks of ``inp`` (world * out.numel() elements, rank-major).  Moves
        the same bytes per link as half an all-reduce.  Under gloo: an all-reduce of a
        host copy, then the chunk."""
        self.reduce_scatter_async(out, inp).wait()
        return out

    def reduce_scatter_async(self, out: torch.Tensor, inp: torch.Tensor):
        """reduce_scatter_ issued in the background: the one-shot xGMI kernel on the side
        stream, or on RCCL's own stream (async_op); gloo completes it here."""
        if self.world_size == 1:
            LocalComm.reduce_scatter_(self, out, inp)
            return _DONE
        m = out.numel()
        if inp.numel() != m * self.world_size:
            raise ValueError(f"reduce_scatter_: {inp.numel()} != {self.world_size} x {m}")
        self._rec("reduce_scatter", inp, out)
        xg = self._xgmi_for(inp)
        if xg is not None:
            ok, h = self._on_side(lambda: xg.reduce_scatter(out, inp, overlap=True))
            if ok:
                return h
        if self.backend == "nccl" and inp.is_cuda and out.is_contiguous() and inp.is_contiguous():
            return self._dist.reduce_scatter_tensor(out, inp, group=self.group, async_op=True)
        host = inp.reshape(-1).cpu()
        self._dist.all_reduce(host, group=self.group)
        out.copy_(host[self.rank * m:(self.rank + 1) * m].view_as(out))
        return _DONE

    def all_gather_into_(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """One all-gather into the rank-major ``out`` (world * inp.numel() elements)."""
        self.all_gather_into_async(out, inp).wait()
        return out

    def all_gather_into_async(self, out: torch.Tensor, inp: torch.Tensor):
        """all_gather_into_ issued in the background (see reduce_scatter_async)."""
        if self.world_size == 1:
            LocalComm.all_gather_into_(self, out, inp)
            return _DONE
        m = inp.numel()
        if out.numel() != m * self.world_size:
            raise ValueError(f"all_gather_into_: {out.numel()} != {self.world_size} x {m}")
        self._rec("all_gather", inp, out)
        xg = self._xgmi_for(inp, any_dtype=True)
        if xg is not None:
            ok, h = self._on_side(lambda: xg.all_gather(out, inp, overlap=True))
            if ok:
                return h
        if self.backend == "nccl" and inp.is_cuda and out.is_contiguous() and inp.is_contiguous():
            return self._dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True)
        # gloo: as raw bytes (it has no int16 / bfloat16 all-gather)
        src = inp.reshape(-1).cpu().contiguous().view(torch.uint8)
        parts = [torch.empty(src.numel(), dtype=torch.uint8) for _ in range(self.world_size)]
        self._dist.all_gather(parts, src, group=self.group)
        out.reshape(-1).copy_(torch.cat(parts).view(inp.dtype))
        return _DONE

    def send_object(self, obj, dst: int) -> None:
        """Point-to-point: ``obj`` to rank ``dst`` (which must call recv_object(src=me))."""
        self._dist.send_object_list([obj], dst=dst, group=self.group)

    # bounded point-to-point array transfer (sharded prepare's row blocks to the writer)
    _DTYPES = ("<f4", "<f8", "<i4", "<i8", "|u1", "<u4", "<u8", "|b1", "<i2", "<u2", "|i1")
    max_msg_bytes = 0           # largest single message sent so far (tests, logging)

    def _p2p(self, t: torch.Tensor, peer: int, send: bool) -> torch.Tensor:
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" \
            else torch.device("cpu")
        x = t.to(dev) if t.device != dev else t
        if send:
            self._dist.send(x.contiguous(), dst=peer, group=self.group)
            return t
        self._dist.recv(x, src=peer, group=self.group)
        return x.cpu() if x.device != t.device else x

    def send_array(self, arr, dst: int, chunk_bytes: int = 1 << 30) -> None:
        """``arr`` (numpy) to rank ``dst`` as a fixed-size header and payload messages of at
        most ``chunk_bytes`` each (recv_array on the peer) -- never one message of the
        whole block (a pickled row block of a 10M-cell shard would be tens of GB)."""
        import numpy as np

        a = np.ascontiguousarray(arr)
        code = self._DTYPES.index(a.dtype.str)
        if a.ndim > 4:
            raise ValueError("send_array: at most 4 dimensions")
        shp = list(a.shape) + [0] * (4 - a.ndim)
        hdr = torch.tensor([a.ndim] + shp + [code, a.nbytes, int(chunk_bytes)], dtype=torch.int64)
        self._p2p(hdr, dst, True)
        raw = torch.from_numpy(a.reshape(-1).view(np.uint8)) if a.nbytes else None
        for o in range(0, a.nbytes, int(chunk_bytes)):
            piece = raw[o:o + int(chunk_bytes)]
            self.max_msg_bytes = max(self.max_msg_bytes, piece.numel())
            self._p2p(piece, dst, True)

    def recv_array(self, src: int):
        """The array rank ``src`` sends with send_array."""
        import numpy as np

        hdr = self._p2p(torch.zeros(8, dtype=torch.int64), src, False).tolist()
        nd, shp, code, nbytes, cb = hdr[0], hdr[1:1 + hdr[0]], hdr[5], hdr[6], hdr[7]
        out = np.empty(nbytes, dtype=np.uint8)
        ot = torch.from_numpy(out)
        for o in range(0, nbytes, cb):
            n = min(cb, nbytes - o)
            ot[o:o + n].copy_(self._p2p(torch.empty(n, dtype=torch.uint8), src, False))
        return out.view(np.dtype(self._DTYPES[code])).reshape(shp)

    def recv_object(self, src: int):
        """Point-to-point: the object rank ``src`` sends with send_object."""
        box = [None]
        self._dist.recv_object_list(box, src=src, group=self.group)
        return box[0]

    def gather_object(self, obj, dst: int = 0):
        """Python objects of every rank on ``dst`` (list in rank order), None elsewhere."""
        if self.world_size == 1:
            return [obj]
        out = [None] * self.world_size if self.rank == dst else None
        self._dist.gather_object(obj, out, dst=dst, group=self.group)
        return out


class EmulatedComm(LocalComm):
    """Rank 0 of a ``world``-rank cell-sharded (DP) solve, run alone on one GPU: every
    collective is replaced by a device copy of the bytes it would deliver, scaled as if
    every rank had contributed this rank's statistics (homogeneous shards).  The solver
    then runs exactly rank 0's per-step work -- the same kernels, shapes and pass counts
    -- so its step time is the per-rank compute time of the real N-GPU job, collectives
    excluded (bench.py --mode dp --emulate-world N; their volume is reported beside it).
    Never used to produce results."""

    def __init__(self, world: int):
        self.rank = 0
        self.world_size = int(world)
        self.bytes = 0          # collective payload bytes issued (per rank)
        # collective launches by kind, and per launch (kind, payload bytes) in order
        self.calls = {"all_reduce": 0, "reduce_scatter": 0, "all_gather": 0}
        self.log: list = []
        self._scratch = None

    def _count(self, kind: str, nbytes: int) -> None:
        self.calls[kind] += 1
        self.bytes += nbytes
        self.log.append((kind, int(nbytes)))

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    def _copy(self, t: torch.Tensor) -> None:
        n = t.numel()
        if self._scratch is None or self._scratch.numel() < n or self._scratch.dtype != t.dtype \
                or self._scratch.device != t.device:
            self._scratch = torch.empty(max(n, 1 << 20), dtype=t.dtype, device=t.device)
        self._scratch[:n].copy_(t.reshape(-1))

    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        self._copy(t)
        self._count("all_reduce", t.numel() * t.element_size())
        if t.is_floating_point():
            t.mul_(self.world_size)
        return t

    def allreduce_scalar(self, v: float) -> float:
        return float(v) * self.world_size

    def reduce_scatter_(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        self._count("reduce_scatter", inp.numel() * inp.element_size())
        out.copy_(inp.reshape(-1)[:out.numel()].view_as(out))
        out.mul_(self.world_size)
        return out

    def all_gather_into_(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        m = inp.numel()
        self._count("all_gather", out.numel() * out.element_size())
        flat = out.reshape(-1)
        for r in range(self.world_size):
            flat[r * m:(r + 1) * m].copy_(inp.reshape(-1))
        return out
