"""Probe: factorize stage wall time with and without early replicate writes
(CNMF_EARLY_WRITE), alternating in ONE process on the e2e bench's data (PBMC scale,
K=5..13 x 100), outputs removed between runs."""
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pandas as pd  # noqa: E402

from cnmf_torch_amd import cNMF  # noqa: E402
from cnmf_torch_amd.utils.anndata_lite import AnnData  # noqa: E402
from cnmf_torch_amd.utils.h5ad import write_h5ad  # noqa: E402
from cnmf_torch_amd.utils.synthetic import simulate_counts  # noqa: E402

d = tempfile.mkdtemp()
X, cells, genes = simulate_counts(10000, 8000, 10, seed=0, sparse=True)
counts = os.path.join(d, "counts.h5ad")
write_h5ad(counts, AnnData(X=X, obs=pd.DataFrame(index=cells), var=pd.DataFrame(index=genes)))
obj = cNMF(output_dir=d, name="p")
obj.prepare(counts, components=list(range(5, 14)), n_iter=100, seed=14, num_highvar_genes=2000)
tmp = os.path.join(d, "p", "cnmf_tmp")
for i, flag in enumerate(["1", "0"] * 4):
    os.environ["CNMF_EARLY_WRITE"] = flag
    for f in os.listdir(tmp):
        if ".spectra.k_" in f and ".iter_" in f or f.endswith(".jsonl"):
            os.remove(os.path.join(tmp, f))
    t0 = time.perf_counter()
    obj.factorize(verbose=False)
    print(f"run {i} early={flag}: factorize {1e3 * (time.perf_counter() - t0):.1f} ms",
          flush=True)
shutil.rmtree(d)
