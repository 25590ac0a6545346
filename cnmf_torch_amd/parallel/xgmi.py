"""One-shot all-reduce over xGMI peer memory.

The cell-sharded DP solver all-reduces one flat float32 buffer per online step (the
``[dB | dA]`` sufficient statistics, a few MB).  RCCL runs that as a ring: 2 (W-1) latency
steps and every byte crossing 2 (W-1)/W links.  On an MI355X node every GPU has a direct
xGMI link to each of the 7 others, so here every rank instead maps the other ranks'
workspaces (``hipIpcOpenMemHandle``) and ONE kernel per call
(``csrc/kernels/xgmi_allreduce.hip``) stages the local buffer, raises a per-slice flag in
every peer, and sums the peers' slices in rank order straight from their HBM -- each byte
crosses one link once, all 7 links at the same time, with one flag handshake per slice.
The sum is in rank order on every rank, so all ranks hold bitwise identical results.

Opt in with ``CNMF_ALLREDUCE=xgmi`` (``DistComm`` then routes float32 device buffers of
up to ``cap`` floats here and everything else to RCCL).  All ranks must be on
one node, each on its own GPU -- or, for tests, several processes on one GPU.  A peer that
never arrives raises the kernel's timeout flag instead of hanging the GPU;
:meth:`XgmiAllReduce.check` turns that into an exception.

The reference has no counterpart: its workers only meet through files
(``/root/reference/src/cnmf/cnmf.py:895-920``, combine).
"""
from __future__ import annotations

import os

import torch

DEFAULT_CAP = 1 << 22            # floats per parity (16 MB): the K=10..20 DP statistics
DEFAULT_TIMEOUT_MS = 10_000


def _hip():
    from .. import ops

    return ops._require_native()


class XgmiTimeout(RuntimeError):
    pass


class XgmiUnavailable(RuntimeError):
    """Some rank could not allocate or export a coherent workspace: every rank raises it
    (the decision is taken collectively), and DistComm stays on RCCL."""


class XgmiAllReduce:
    """Peer-mapped workspaces of every rank of ``group`` and the one-shot reduce.

    Collective: every rank constructs it (exchanging IPC handles through ``group``, which
    may be gloo or RCCL), then every rank issues the same sequence of :meth:`__call__`.
    """

    def __init__(self, group=None, device: torch.device | None = None,
                 cap: int | None = None, timeout_ms: int | None = None,
                 blocks: int | None = None):
        import torch.distributed as dist

        hip = _hip()
        self._dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > hip.xgmi_max_ranks():
            raise ValueError(f"xgmi all-reduce handles up to {hip.xgmi_max_ranks()} ranks")
        self.device = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
        cap = int(cap if cap is not None else DEFAULT_CAP)
        self.cap = -(-cap // 4) * 4
        self.blocks = int(blocks or min(hip.xgmi_max_blocks(),
                                        max(1, hip.cu_count(self.device.index or 0) // 2)))
        ms = int(timeout_ms if timeout_ms is not None else DEFAULT_TIMEOUT_MS)
        self.limit = int(hip.xgmi_wall_clock_khz(self.device.index or 0)) * max(1, ms)
        # Workspace memory: uncached (or fine-grained) device memory, never coarse-grained
        # hipMalloc -- peers hand data over INSIDE a kernel, across GPUs, and only those
        # kinds are coherent across devices while kernels run (xgmi_allreduce.hip,
        # cnmf_xgmi_alloc).  Every rank reports success or its error and all ranks take
        # the same decision, so a refusal on one rank cannot strand the others in a
        # collective.
        self._base, self.alloc_flags, handle, err = 0, 0, None, None
        try:
            with torch.cuda.device(self.device):
                self._base, self.alloc_flags = hip.xgmi_alloc(self.cap)
                handle = hip.xgmi_handle(self._base)
        except RuntimeError as e:            # refused flag / IPC export on this rank
            err = f"rank {self.rank}: {e}"
        handles = [None] * self.world
        dist.all_gather_object(handles, (handle, err), group=group)
        errors = [e_ for _, e_ in handles if e_ is not None]
        if errors:
            if self._base:
                with torch.cuda.device(self.device):
                    hip.xgmi_free(self._base)
            self.closed = True
            raise XgmiUnavailable("; ".join(errors))
        handles = [h_ for h_, _ in handles]
        self._opened = []
        peers = []
        with torch.cuda.device(self.device):
            for r, h in enumerate(handles):
                if r == self.rank:
                    peers.append(self._base)
                else:
                    p = hip.xgmi_open(h)
                    self._opened.append(p)
                    peers.append(p)
        self.peers = torch.tensor(peers, dtype=torch.int64, device=self.device)
        self.timeout = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.epoch = 0
        self.closed = False
        # nobody's first flag store may land before every rank has mapped every workspace
        dist.barrier(group=group)

    @property
    def memory_kind(self) -> str:
        """'uncached' or 'fine-grained': the allocation flags of this rank's workspace as
        hipPointerGetAttributes reports them (never coarse-grained)."""
        hip = _hip()
        f = hip.ptr_alloc_flags(self._base)
        return {hip.MALLOC_UNCACHED: "uncached", hip.MALLOC_FINEGRAINED: "fine-grained"}.get(
            f, f"flags={f:#x}")

    def supports(self, t: torch.Tensor) -> bool:
        return (not self.closed and t.device == self.device and t.dtype == torch.float32
                and t.is_contiguous() and t.numel() <= self.cap)

    def __call__(self, t: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """Sum of ``t`` over the ranks into ``out`` (default: in place)."""
        if not self.supports(t):
            raise ValueError("xgmi all-reduce: contiguous float32 on this rank's device, "
                             f"at most {self.cap} elements")
        out = t if out is None else out
        if out.shape != t.shape or not self.supports(out):
            raise ValueError("xgmi all-reduce: out must match t")
        self.epoch = (self.epoch + 1) & 0xFFFFFFFF     # compares are wrap-safe
        from ..ops import _stream_ptr

        _hip().xgmi_allreduce(self.peers.data_ptr(), self.world, self.rank, t.data_ptr(),
                              out.data_ptr(), t.numel(), self.cap, self.epoch, self.limit,
                              self.timeout.data_ptr(), self.blocks, _stream_ptr(t))
        return out

    def check(self) -> None:
        """Raise on EVERY rank if any call so far gave up waiting for a peer on ANY rank
        (host sync; collective).  The flags are max-reduced first: a rank that alone saw
        the timeout would otherwise raise while its peers wait in the next collective."""
        flag = self.timeout.clone()
        self._dist.all_reduce(flag, op=self._dist.ReduceOp.MAX, group=self.group)
        if int(flag.item()) != 0:
            raise XgmiTimeout("xgmi all-reduce: a peer did not arrive within the wait limit "
                              "(mismatched collective sequence or a dead rank); results of "
                              "the calls since are invalid")

    def close(self) -> None:
        """Collective teardown: no rank unmaps or frees while another may still read."""
        if self.closed:
            return
        torch.cuda.synchronize(self.device)
        self._dist.barrier(group=self.group)
        hip = _hip()
        with torch.cuda.device(self.device):
            for p in self._opened:
                hip.xgmi_close(p)
            self._opened = []
            torch.cuda.synchronize(self.device)
        self._dist.barrier(group=self.group)
        with torch.cuda.device(self.device):
            hip.xgmi_free(self._base)
        self.closed = True


def wanted() -> bool:
    return os.environ.get("CNMF_ALLREDUCE", "rccl").lower() == "xgmi"
