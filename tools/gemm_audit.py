"""Audit: every library-GEMM call (torch matmul family) the k-selection and consensus
stages make on the device, with its shapes, dtype and the calling line in the package --
the list that must be empty for "no library GEMM in consensus" (SURVEY.md H4-H6).

    python tools/gemm_audit.py [--cells 10000 --genes 8000 --kmin 5 --kmax 13]

Runs prepare -> factorize -> combine on the e2e bench's synthetic data, then
k_selection_plot and consensus under a TorchFunctionMode that records mm / matmul / bmm /
addmm / einsum / linalg calls on device tensors.  Prints one JSON line.
"""
import argparse
import collections
import json
import os
import sys
import tempfile
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import pandas as pd  # noqa: E402
import torch  # noqa: E402
from torch.overrides import TorchFunctionMode  # noqa: E402

from cnmf_torch_amd import cNMF  # noqa: E402
from cnmf_torch_amd.utils.anndata_lite import AnnData  # noqa: E402
from cnmf_torch_amd.utils.h5ad import write_h5ad  # noqa: E402
from cnmf_torch_amd.utils.synthetic import simulate_counts  # noqa: E402

_GEMMS = {"mm", "matmul", "bmm", "addmm", "addbmm", "baddbmm", "einsum", "__matmul__",
          "__rmatmul__", "mv", "addmv", "dot", "tensordot", "lstsq", "solve", "cholesky",
          "eigh", "svd", "qr", "inv"}


class _Audit(TorchFunctionMode):
    def __init__(self):
        super().__init__()
        self.calls = collections.Counter()

    def __torch_function__(self, func, types, args=(), kwargs=None):
        name = getattr(func, "__name__", str(func))
        if name in _GEMMS:
            ts = [a for a in args if isinstance(a, torch.Tensor)]
            if any(t.is_cuda for t in ts):
                where = "?"
                for fr in reversed(traceback.extract_stack()[:-1]):
                    if "cnmf_torch_amd" in fr.filename:
                        where = f"{os.path.basename(fr.filename)}:{fr.lineno}"
                        break
                key = (name, where, str(ts[0].dtype), " x ".join(str(tuple(t.shape)) for t in ts))
                self.calls[key] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=10000)
    ap.add_argument("--genes", type=int, default=8000)
    ap.add_argument("--hvg", type=int, default=2000)
    ap.add_argument("--kmin", type=int, default=5)
    ap.add_argument("--kmax", type=int, default=13)
    ap.add_argument("--n-iter", type=int, default=100)
    a = ap.parse_args()
    work = tempfile.mkdtemp(prefix="cnmf_audit_")
    X, cells, genes = simulate_counts(a.cells, a.genes, 9, seed=0, sparse=True)
    counts = os.path.join(work, "counts.h5ad")
    write_h5ad(counts, AnnData(X=X, obs=pd.DataFrame(index=cells), var=pd.DataFrame(index=genes)))
    ks = list(range(a.kmin, a.kmax + 1))
    obj = cNMF(output_dir=work, name="audit")
    obj.prepare(counts, components=ks, n_iter=a.n_iter, seed=14, num_highvar_genes=a.hvg,
                prewarm=False)
    obj.factorize(verbose=False)
    obj.combine()
    out = {}

    def kstats():   # k_selection_plot's per-K statistics, serially (the stage runs them on
        for k in ks:  # worker threads, which a TorchFunctionMode does not follow)
            obj.consensus(k, skip_density_and_return_after_stats=True, show_clustering=False,
                          close_clustergram_fig=True)

    for stage, fn in (("k_selection_stats", kstats),
                      ("consensus", lambda: obj.consensus(ks[len(ks) // 2], density_threshold=0.1,
                                                          show_clustering=True,
                                                          close_clustergram_fig=True))):
        with _Audit() as au:
            fn()
        out[stage] = [{"op": k[0], "at": k[1], "dtype": k[2], "shapes": k[3], "calls": n}
                      for k, n in au.calls.most_common()]
    print(json.dumps({"metric": "library GEMM calls on the device per stage",
                      "device": torch.cuda.get_device_name(0) if torch.cuda.is_available()
                      else "cpu", "stages": out}))


if __name__ == "__main__":
    main()
