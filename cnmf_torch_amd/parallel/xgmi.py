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
        # a collective issued to OVERLAP compute (DistComm's async reduce-scatter /
        # all-gather under the DP step's cooperative solves) spins inside the kernel until
        # its peers arrive; its blocks must fit the CUs the cooperative solves' co-residency
        # budget leaves free (ops._coop_resident keeps COOP_MARGIN_CUS), or a solve's
        # workgroups could wait on siblings that cannot be placed
        from ..ops import COOP_MARGIN_CUS

        self.overlap_blocks = max(1, min(self.blocks, COOP_MARGIN_CUS))
        # every launch runs on this ONE stream (ordered behind the caller's): the calls
        # share the device epoch counter and the two staging parities
        self.stream = torch.cuda.Stream(device=self.device)
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
        # the call counter lives on the device (advanced by each launch's last block), so
        # the collectives replay correctly from a captured HIP graph
        self.ep = torch.zeros(2, dtype=torch.int32, device=self.device)   # [epoch, arrivals]
        self.epoch = 0          # host-side count of calls issued (diagnostics)
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

    @staticmethod
    def _f32(t: torch.Tensor) -> torch.Tensor | None:
        """A contiguous device buffer as float32 words (byte / int16 payloads of the DP
        step travel as their bit patterns), or None."""
        if not t.is_contiguous():
            return None
        if t.dtype == torch.float32:
            return t.reshape(-1)
        nb = t.numel() * t.element_size()
        if nb % 4 or t.data_ptr() % 4:
            return None
        return t.reshape(-1).view(torch.uint8).view(torch.float32)

    def _launch(self, mode: int, src: torch.Tensor, dst: torch.Tensor, m: int,
                overlap: bool = False) -> None:
        # every collective shares one device epoch counter and two staging parities, which
        # is only sound when all launches are ordered on one stream: a call from another
        # stream forks onto self.stream and joins back (also inside a graph capture)
        cur = torch.cuda.current_stream(self.device)
        fork = cur.cuda_stream != self.stream.cuda_stream
        if fork:
            self.stream.wait_stream(cur)
        self.epoch += 1
        e = self.ep
        _hip().xgmi_collective(mode, self.peers.data_ptr(), self.world, self.rank,
                               src.data_ptr(), dst.data_ptr(), int(m), self.cap, 0,
                               e.data_ptr(), e.data_ptr() + 4, self.limit,
                               self.timeout.data_ptr(),
                               self.overlap_blocks if overlap else self.blocks,
                               self.stream.cuda_stream)
        if fork:      # (the caller's stream waits: its later frees of src / dst are safe)
            cur.wait_stream(self.stream)

    def __call__(self, t: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """Sum of ``t`` over the ranks into ``out`` (default: in place)."""
        if not self.supports(t):
            raise ValueError("xgmi all-reduce: contiguous float32 on this rank's device, "
                             f"at most {self.cap} elements")
        out = t if out is None else out
        if out.shape != t.shape or not self.supports(out):
            raise ValueError("xgmi all-reduce: out must match t")
        self._launch(0, t, out, t.numel())
        return out

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, overlap: bool = False) -> bool:
        """out = chunk ``rank`` of the rank-ordered sum of ``inp`` (world equal chunks,
        rank-major): each rank reads only its chunk from every peer -- one hop per link.
        float32 only (a sum).  Returns False when the buffers do not qualify."""
        if self.closed or inp.dtype != torch.float32 or out.dtype != torch.float32 or \
                inp.device != self.device or out.device != self.device or \
                not (inp.is_contiguous() and out.is_contiguous()) or \
                inp.numel() != out.numel() * self.world or inp.numel() > self.cap:
            return False
        self._launch(1, inp, out, out.numel(), overlap)
        return True

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, overlap: bool = False) -> bool:
        """out (world equal chunks, rank-major) = every rank's ``inp``; any dtype whose
        buffers are whole 4-byte words.  Returns False when the buffers do not qualify."""
        src, dst = self._f32(inp), self._f32(out)
        if self.closed or src is None or dst is None or inp.device != self.device or \
                out.device != self.device or dst.numel() != src.numel() * self.world or \
                src.numel() > self.cap:
            return False
        self._launch(2, src, dst, src.numel(), overlap)
        return True

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
