"""Figures: consensus clustergram (C25, cnmf.py:1160-1253), K-selection plot (C27,
cnmf.py:1311-1332) and the Preprocess QC histograms (C32).  matplotlib, Agg backend.

Figures that the caller closes anyway (``close=True``: CLI and pipeline runs) can be drawn
by :class:`PlotWorker`, a child Python process started when the first such stage begins:
it imports matplotlib (~0.8 s on a fresh box, where its .pyc files are compiled) while the
stage computes on the GPU, then draws the same figure with the same code, and stays up for
the following stages.  This module imports
only numpy at the top (pandas objects are only passed in by the API), so the worker
never loads torch or pandas or touches the GPU.
"""
from __future__ import annotations

import atexit
import concurrent.futures as cf
import itertools
import json
import os
import struct
import subprocess
import sys
import tempfile
import threading
import time
import zlib

import numpy as np


def _plt():
    import matplotlib

    if matplotlib.get_backend().lower() not in ("agg", "module://matplotlib_inline.backend_inline"):
        try:
            matplotlib.use("Agg")
        except Exception:
            pass
    import matplotlib.pyplot as plt

    return plt


def _leaf_order(dist: np.ndarray, labels: pd.Series) -> list[int]:
    """Clusters in label order; spectra inside a cluster by average-linkage leaves."""
    from scipy.cluster.hierarchy import leaves_list, linkage
    from scipy.spatial.distance import squareform

    order: list[int] = []
    lab = labels.values
    for cl in sorted(set(lab)):
        members = np.flatnonzero(lab == cl)
        if members.size > 1:
            sub = squareform(dist[np.ix_(members, members)], checks=False)
            sub[sub < 0] = 0
            order += list(members[leaves_list(linkage(sub, "average"))])
        else:
            order += list(members)
    return order


def clustergram(dist: np.ndarray, labels: pd.Series, local_density: pd.DataFrame | None,
                density_filter: np.ndarray | None, density_threshold: float, path: str,
                close: bool = False):
    from matplotlib import gridspec

    plt = _plt()
    order = _leaf_order(dist, labels)
    D = dist[np.ix_(order, order)]
    widths, heights = [0.5, 9, 0.5, 4, 1], [0.5, 9]
    fig = plt.figure(figsize=(sum(widths), sum(heights)))
    gs = gridspec.GridSpec(2, 5, fig, 0.01, 0.01, 0.98, 0.98, height_ratios=heights,
                           width_ratios=widths, wspace=0, hspace=0)
    ax = fig.add_subplot(gs[1, 1], xticks=[], yticks=[])
    # the heatmap colour-mapped once at its own 900 x 900 size, then drawn as RGBA: Agg
    # resamples an RGBA image without re-mapping the ~5 M output pixels through the
    # colormap (the same nearest-pixel picture); the colour bar keeps the scalar mapping
    from matplotlib import cm, colors

    norm = colors.Normalize(vmin=float(D.min()), vmax=float(D.max()))
    im = cm.ScalarMappable(norm=norm, cmap="viridis")
    ax.imshow(im.to_rgba(D, bytes=True), interpolation="none", aspect="auto",
              rasterized=True)
    lab = labels.values[order]
    left = fig.add_subplot(gs[1, 0], xticks=[], yticks=[])
    left.imshow(lab.reshape(-1, 1), interpolation="none", cmap="Spectral", aspect="auto",
                rasterized=True)
    top = fig.add_subplot(gs[0, 1], xticks=[], yticks=[])
    top.imshow(lab.reshape(1, -1), interpolation="none", cmap="Spectral", aspect="auto",
               rasterized=True)
    hgs = gridspec.GridSpecFromSubplotSpec(3, 1, subplot_spec=gs[1, 3], wspace=0, hspace=0)
    hax = fig.add_subplot(hgs[0, 0], title="Local density histogram")
    if local_density is not None:
        hax.hist(local_density.values, bins=np.linspace(0, 1, 50))
    hax.yaxis.tick_right()
    xl, yl = hax.get_xlim(), hax.get_ylim()
    if density_threshold < xl[1]:
        hax.axvline(density_threshold, linestyle="--", color="k")
        hax.text(density_threshold + 0.02, yl[1] * 0.95, "filtering\nthreshold\n\n", va="top")
    hax.set_xlim(xl)
    if density_filter is not None:
        removed = int((~density_filter).sum())
        hax.set_xlabel("Mean distance to k nearest neighbors\n\n%d/%d (%.0f%%) spectra above "
                       "threshold\nwere removed prior to clustering"
                       % (removed, len(density_filter), 100 * removed / max(len(density_filter), 1)))
    cgs = gridspec.GridSpecFromSubplotSpec(8, 1, subplot_spec=hgs[1, 0], wspace=0, hspace=0)
    cax = fig.add_subplot(cgs[4, 0], title="Euclidean Distance")
    fig.colorbar(im, cax=cax, ticks=np.linspace(float(D.min()), float(D.max()), 3),
                 orientation="horizontal")
    _save(fig, path)
    if close:
        plt.close(fig)
    return fig


def _png_chunk(tag: bytes, data: bytes) -> bytes:
    return (struct.pack(">I", len(data)) + tag + data
            + struct.pack(">I", zlib.crc32(data, zlib.crc32(tag)) & 0xFFFFFFFF))


def write_png_rgba(path: str, rgba: np.ndarray, dpi: float, threads: int = 8) -> None:
    """RGBA8 PNG of ``rgba`` (H, W, 4) with the deflate stream compressed in row bands on
    ``threads`` threads (native, csrc/io/npzio.cpp; this Python form is the fallback when
    the module is not built).  Each band ends in a full flush, so the concatenated raw
    deflate blocks are one valid stream -- the pigz construction.  Same
    chunks as matplotlib's Agg/PIL output (IHDR, pHYs from ``dpi``, a Software tEXt, IDAT,
    IEND) and the same pixels; filter 0 on every row, zlib level 1.  The clustergram
    (3750 x 2375) encoded in ~0.45 s through PIL."""
    import matplotlib

    software = f"Matplotlib version{matplotlib.__version__}, https://matplotlib.org/"
    try:
        from . import _npzio
    except ImportError:
        _npzio = None
    if _npzio is not None and hasattr(_npzio, "write_png_rgba"):
        # native: the bands deflate on std::threads (Python 3.10's zlib holds the GIL)
        _npzio.write_png_rgba(path, np.ascontiguousarray(rgba), float(dpi), software, 1,
                              int(threads))
        return
    h, w, _ = rgba.shape
    raw = np.empty((h, 1 + 4 * w), dtype=np.uint8)
    raw[:, 0] = 0
    raw[:, 1:] = rgba.reshape(h, 4 * w)
    band = max(1, -(-h // max(1, threads)))
    pieces = [raw[a:a + band] for a in range(0, h, band)]

    def deflate(i):
        co = zlib.compressobj(1, zlib.DEFLATED, -15)
        out = co.compress(pieces[i].tobytes())
        return out + co.flush(zlib.Z_FINISH if i == len(pieces) - 1 else zlib.Z_FULL_FLUSH)

    with cf.ThreadPoolExecutor(max_workers=len(pieces)) as ex:
        body = b"".join(ex.map(deflate, range(len(pieces))))
    adler = 1
    for pc in pieces:
        adler = zlib.adler32(pc, adler)
    idat = b"\x78\x01" + body + struct.pack(">I", adler & 0xFFFFFFFF)
    ppm = int(round(dpi / 0.0254))
    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(_png_chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)))
        f.write(_png_chunk(b"pHYs", struct.pack(">IIB", ppm, ppm, 1)))
        f.write(_png_chunk(b"tEXt", b"Software\x00" + software.encode()))
        f.write(_png_chunk(b"IDAT", idat))
        f.write(_png_chunk(b"IEND", b""))


def _save(fig, path: str) -> None:
    """Atomic PNG write (temp file in the destination directory + rename)."""
    d = os.path.dirname(os.path.abspath(path)) or "."
    fd, tmp = tempfile.mkstemp(prefix=".tmp_" + os.path.basename(path) + ".", suffix=".png",
                               dir=d)
    os.close(fd)
    try:
        # dpi 250 as cnmf.py:1251.  The Agg canvas renders at that dpi and the PNG is
        # encoded on several threads (write_png_rgba): PIL's single-threaded encode of the
        # 3750 x 2375 clustergram was ~0.45 s of its ~1.5 s
        if fig.canvas.get_default_filetype() == "png" and \
                type(fig.canvas).__name__ == "FigureCanvasAgg":
            old = fig.get_dpi()
            fig.set_dpi(250)
            try:
                fig.canvas.draw()
                write_png_rgba(tmp, np.asarray(fig.canvas.buffer_rgba()), 250)
            finally:
                fig.set_dpi(old)
        else:
            fig.savefig(tmp, dpi=250, pil_kwargs={"compress_level": 1})
        os.replace(tmp, path)
    except BaseException:
        if os.path.exists(tmp):
            os.remove(tmp)
        raise


def k_selection(stats: pd.DataFrame, path: str, close: bool = False):
    plt = _plt()
    fig = plt.figure(figsize=(6, 4))
    ax1 = fig.add_subplot(111)
    ax2 = ax1.twinx()
    ax1.plot(stats.k, stats.silhouette, "o-", color="b")
    ax1.set_ylabel("Stability", color="b", fontsize=15)
    for t in ax1.get_yticklabels():
        t.set_color("b")
    ax2.plot(stats.k, stats.prediction_error, "o-", color="r")
    ax2.set_ylabel("Error", color="r", fontsize=15)
    for t in ax2.get_yticklabels():
        t.set_color("r")
    ax1.set_xlabel("Number of Components", fontsize=15)
    ax1.grid(True)
    plt.tight_layout()
    _save(fig, path)
    if close:
        plt.close(fig)
    return fig


def count_hist(X, num_cells: int = 1000, title="Quantile thresholded normalized count distribution"):
    import scipy.sparse as sp

    plt = _plt()
    z = X[:num_cells]
    z = z.toarray() if sp.issparse(z) else np.asarray(z)
    y = z.reshape(-1)
    fig, ax = plt.subplots()
    ax.hist(y[y > 0], bins=100)
    ax.set_title(title)
    return fig


class _PlotProc:
    """The figure-drawing child process, shared by every PlotWorker of this process: it
    imports matplotlib once (~0.8-1 s on a fresh box), then draws job after job, and
    acknowledges each on stdout ("ok <id>" / "err <id>").  Closed at interpreter exit."""

    _inst = None
    _lock = threading.Lock()

    def __init__(self):
        env = dict(os.environ, MPLBACKEND="Agg", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "plot_worker.py")
        self.proc = subprocess.Popen([sys.executable, script], stdin=subprocess.PIPE,
                                     stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                                     env=env, text=True, bufsize=1)
        self.acks: dict = {}
        self.alive = True
        self.cv = threading.Condition()
        self.reader = threading.Thread(target=self._read, daemon=True)
        self.reader.start()

    def _read(self) -> None:
        try:
            for line in self.proc.stdout:
                parts = line.split()
                if len(parts) == 2 and parts[0] in ("ok", "err"):
                    with self.cv:
                        self.acks[int(parts[1])] = parts[0] == "ok"
                        self.cv.notify_all()
        finally:
            with self.cv:
                self.alive = False
                self.cv.notify_all()

    def send(self, job: dict) -> bool:
        try:
            self.proc.stdin.write(json.dumps(job) + "\n")
            self.proc.stdin.flush()
            return True
        except Exception:
            return False

    def result(self, jid: int, deadline: float):
        """True / False once job ``jid`` is acknowledged; None if the child died or the
        deadline passed first."""
        with self.cv:
            while jid not in self.acks and self.alive:
                left = deadline - time.monotonic()
                if left <= 0 or not self.cv.wait(timeout=left):
                    if jid not in self.acks:
                        return None
            return self.acks.pop(jid, None)

    def close(self) -> None:
        try:
            self.proc.stdin.close()
            self.proc.wait(timeout=10)
        except Exception:
            self.proc.kill()

    @classmethod
    def get(cls) -> "_PlotProc":
        with cls._lock:
            if cls._inst is None or not cls._inst.alive or cls._inst.proc.poll() is not None:
                cls._inst = cls()
                atexit.register(cls._inst.close)
                # atexit runs last-registered first: deferred figures are finished while
                # the child is still up, then it is closed
                atexit.register(flush_figures)
            return cls._inst


def prestart() -> None:
    """Start the shared figure process now (it imports matplotlib while the caller
    computes), unless this process already imported pyplot."""
    if "matplotlib.pyplot" in sys.modules:
        return
    try:
        _PlotProc.get()
    except Exception:
        pass                       # figures then start their child (or draw) on demand


class PlotWorker:
    """Out-of-process figure drawer (see the module docstring).  ``submit`` hands one
    figure job to the shared child (arrays through a temporary .npz); ``wait`` blocks until
    the child has written this worker's figures.  The child stays up for the next stage
    (k_selection_plot then consensus import matplotlib once).  Any failure of the child
    falls back to drawing in this process, so figures are never lost."""

    _ids = itertools.count()

    def __init__(self):
        self.proc = _PlotProc.get()
        self.jobs = []

    def submit(self, kind: str, path: str, **arrays) -> None:
        fd, npz = tempfile.mkstemp(suffix=".npz")
        os.close(fd)
        np.savez(npz, **{k: np.asarray(v) for k, v in arrays.items()})
        jid = next(self._ids)
        sent = self.proc.send({"id": jid, "kind": kind, "path": path, "npz": npz})
        self.jobs.append((jid, kind, path, npz, sent))

    def wait(self, timeout: float = 300.0, defer: bool = False) -> None:
        """Block until this worker's figures are written (drawing any the child failed
        here).  ``defer``: return at once and finish them in :func:`flush_figures` (the
        CLI calls it before exiting, and it runs at interpreter exit), so a figure renders
        while the caller's next stage computes."""
        if defer:
            if self.jobs:
                with _DEFER_LOCK:
                    _DEFERRED.append(self)
            return
        deadline = time.monotonic() + timeout
        for jid, kind, path, npz, sent in self.jobs:
            ok = sent and self.proc.result(jid, deadline) is True and os.path.exists(path)
            if not ok:   # draw here instead
                with np.load(npz, allow_pickle=False) as f:
                    draw_job(kind, path, {k: f[k] for k in f.files})
            if os.path.exists(npz):
                os.remove(npz)
        self.jobs = []


_DEFERRED: list = []
_DEFER_LOCK = threading.Lock()


def flush_figures(timeout: float = 300.0) -> None:
    """Finish every figure deferred by ``PlotWorker.wait(defer=True)``."""
    while True:
        with _DEFER_LOCK:
            if not _DEFERRED:
                return
            w = _DEFERRED.pop(0)
        w.wait(timeout)




def draw_job(kind: str, path: str, a: dict) -> None:
    """Draw one PlotWorker job from its arrays (in the worker, or as the fallback).  The
    drawing functions read only ``.k`` / ``.silhouette`` / ``.prediction_error`` and
    ``.values`` of their pandas arguments, so the job passes plain namespaces: the figure
    process never imports pandas (0.6 s of its start-up, profiles/r6j_*)."""
    from types import SimpleNamespace as _NS

    if kind == "k_selection":
        stats = _NS(k=a["k"], silhouette=a["silhouette"],
                    prediction_error=a["prediction_error"])
        k_selection(stats, path, close=True)
    elif kind == "clustergram":
        labels = _NS(values=np.asarray(a["labels"]))
        dens = (_NS(values=np.asarray(a["local_density"]).reshape(-1, 1))
                if a["local_density"].size else None)
        filt = a["density_filter"].astype(bool) if a["density_filter"].size else None
        clustergram(a["dist"], labels, dens, filt, float(a["density_threshold"]), path,
                    close=True)
    else:
        raise ValueError(kind)
