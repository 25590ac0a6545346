"""factorize on the GPU with CNMF_EARLY_WRITE=1 (opt-in): replicates that finish early
are written while the rest of the ragged batch still solves (NMFBatchSolver.run(
on_retire=...), api.factorize_jobs).  The files and their manifest hashes equal the
default write-everything-at-the-end path."""
import json
import os

import numpy as np
import pandas as pd
import pytest

from cnmf_torch_amd import cNMF, load_df_from_npz, save_df_to_npz
from cnmf_torch_amd.utils.synthetic import simulate_counts

pytestmark = pytest.mark.gpu


def _run(tmp, fn, early: str, monkeypatch):
    monkeypatch.setenv("CNMF_EARLY_WRITE", early)
    obj = cNMF(output_dir=str(tmp / f"early{early}"), name="g")
    obj.prepare(fn, components=[4, 5, 6], n_iter=40, seed=5, num_highvar_genes=300,
                batch_size=400)
    obj.factorize(worker_i=0, total_workers=1, verbose=False)
    return obj


def test_early_replicate_writes_equal_end_of_batch_writes(tmp_path, monkeypatch):
    X, cells, genes = simulate_counts(1500, 500, 5, seed=4, sparse=False)
    fn = str(tmp_path / "counts.df.npz")
    save_df_to_npz(pd.DataFrame(X, index=cells, columns=genes), fn)
    a = _run(tmp_path, fn, "1", monkeypatch)
    b = _run(tmp_path, fn, "0", monkeypatch)
    for k in (4, 5, 6):
        for it in range(40):
            fa, fb = a.paths["iter_spectra"] % (k, it), b.paths["iter_spectra"] % (k, it)
            da, db = load_df_from_npz(fa), load_df_from_npz(fb)
            np.testing.assert_array_equal(da.values, db.values)
            assert list(da.columns) == list(db.columns) and list(da.index) == list(db.index)

    def manifest(o):
        recs = [json.loads(l) for l in open(o.paths["replicate_manifest"])]
        return {(r["k"], r["iter"]): r["sha256"] for r in recs}

    ma, mb = manifest(a), manifest(b)
    assert len(ma) == 120 and ma == mb
    assert a.verify_replicates() == []
