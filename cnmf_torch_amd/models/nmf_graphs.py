"""NMFBatchSolver: HIP-graph capture / replay of the online passes per batch layout over a
persistent arena (split out of models/nmf.py)."""
from __future__ import annotations

import collections
import os
import threading

import numpy as np
import torch

from .. import ops
from .nmf_base import log
from .nmf_batch import _Batch


# per host thread: no graph capture (NMFBatchSolver.run_concurrent's workers -- a capture
# in one thread while another thread allocates and frees on its own stream is outside
# what the caching allocator's capture pools guarantee)
_TLS = threading.local()

# pass-graph captures made by this process (bench.py reports those inside its timed region)
CAPTURES = [0]


class _GraphMixin:
    """NMFBatchSolver methods: HIP-graph capture / replay of the online passes per batch
    layout over a persistent arena."""

    # ------------------------------------------------------------------ graphs / arena
    def _graphs_wanted(self, kpos) -> bool:
        """Replay the fused online passes from HIP graphs captured once per batch layout
        and kept across runs (CNMF_GRAPHS: 'auto' (default) = batches of <= 256
        replicates, whose passes are short enough for the host's per-pass enqueue to
        show; '1' any batch; '0' never).  Needs the fused step's preconditions (checked
        again per run by _fused_ok)."""
        env = os.environ.get("CNMF_GRAPHS", "auto")
        o = self.opts
        if env == "0" or self.X.device.type != "cuda" or self.beta != 2.0 or o.mode != "online":
            return False
        if getattr(_TLS, "no_graphs", False):     # run_concurrent's worker threads
            return False
        if env != "1" and len(kpos) > 256:
            return False
        return (o.algo == "mu" and o.online_stats == "pass" and o.online_inner_conv == "loss"
                and not self.comm.is_distributed and int(np.max(kpos)) <= 64
                and os.environ.get("CNMF_FUSED_STEP", "1") != "0"
                and all(v == 0.0 for v in (o.l1_H, o.l2_H, o.l1_W, o.l2_W)))

    def _arena(self, kpos) -> dict:
        """HT / W / state tensors of a batch with this rank vector, kept across runs on the
        current stream (see _Batch's arena)."""
        import collections

        key = (tuple(int(k) for k in kpos), ops._stream_ptr(self.X))
        if not hasattr(self, "_arenas"):
            self._arenas = collections.OrderedDict()
        a = self._arenas.get(key)
        if a is None:
            N, G = self.X.shape
            dev, tot, R = self.X.device, int(np.sum(kpos)), len(kpos)
            sf = torch.zeros((3, R), dtype=torch.float64, device=dev)
            si = torch.zeros((5, R), dtype=torch.int32, device=dev)
            a = {"HT": torch.zeros((tot, N), device=dev, dtype=self.X.dtype),
                 "W": torch.zeros((tot, G), device=dev, dtype=self.X.dtype),
                 "sf": sf, "si": si,
                 "state": {"err_init": sf[0], "err_prev": sf[1], "err": sf[2],
                           "active": si[0], "converged": si[1], "n_pass": si[2]},
                 "h_iters": si[3], "w_iters": si[4],
                 "gate": torch.ones(1, dtype=torch.int32, device=dev),
                 "slots": collections.OrderedDict()}
            self._arenas[key] = a
            while len(self._arenas) > 4:
                self._arenas.popitem(last=False)
        else:
            self._arenas.move_to_end(key)
        return a

    def _slot(self, st: _Batch, steps) -> dict:
        """Per-layout slot of an arena batch: the fused step's workspaces (fixed addresses),
        the solver's capture stream and, once captured, the pass's HIP graph."""
        a = st.arena
        # (a streaming run's pass graph holds its feed's ring / store addresses)
        key = (st.n_act, tuple(int(k) for k in st.kpos[:st.n_act]),
               tuple(tuple(b) for b in steps), st.feed.buf_uid if st.feed is not None else None)
        slots = a["slots"]
        sl = slots.get(key)
        if sl is None:
            sl = {"fb": self._fused_bufs(st, steps), "graph": None, "failed": False,
                  "stream": self._capture_stream()}
            slots[key] = sl
            while len(slots) > 24:
                slots.popitem(last=False)
        else:
            slots.move_to_end(key)
        return sl

    def _capture_stream(self):
        """The one side stream this solver captures pass graphs on (captures are serial,
        the graphs replay on the caller's stream).  One per solver, not one per layout:
        a new HIP stream cost ~0.6 ms of host time at each new layout's first pass
        (hipStreamCreateWithPriority while torch's stream pool fills,
        profiles/r6zl_boundary_gaps.txt)."""
        s = getattr(self, "_cap_stream", None)
        if s is None or s.device != self.X.device:
            s = self._cap_stream = torch.cuda.Stream(self.X.device)
        return s

    def _replay_slot(self, sl: dict, st: _Batch, steps) -> bool:
        """Run one non-final fused pass from the slot's graph (captured on first use, on
        the slot's own stream, from a pass whose operands are already in place).  False:
        capture unavailable -- the caller runs the pass eagerly."""
        if sl["failed"]:
            return False
        if sl["graph"] is None:
            g = torch.cuda.CUDAGraph()
            main = torch.cuda.current_stream(self.X.device)
            o = self.opts
            ops.coop_reserve(self.X.device, sl["stream"].cuda_stream,
                             max(gr.n for gr in st.groups), int(o.online_chunk_max_iter),
                             int(o.inner_check_every))
            sl["stream"].wait_stream(main)
            try:
                with torch.cuda.stream(sl["stream"]):
                    # thread-local capture: run_concurrent's other host threads keep
                    # issuing (and synchronising) their own streams meanwhile
                    g.capture_begin(capture_error_mode="thread_local")
                    try:
                        self._fused_pass(st, steps, sl["fb"], False)
                    finally:
                        g.capture_end()
            except RuntimeError as e:
                sl["failed"] = True
                sl["error"] = str(e)
                log.warning("pass graph capture failed (%s); eager passes for this layout", e)
                return False
            main.wait_stream(sl["stream"])
            sl["graph"] = g
            CAPTURES[0] += 1
        sl["graph"].replay()
        return True
