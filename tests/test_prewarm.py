"""utils.prewarm: the background first-use loading cNMF.prepare starts on a GPU."""
import pytest
import torch

from cnmf_torch_amd.utils import prewarm


def test_prewarm_is_a_noop_off_the_gpu():
    assert prewarm.start("cpu") == []
    prewarm.wait()          # nothing started: returns at once


def test_cli_prepare_turns_prewarm_off(monkeypatch, tmp_path):
    """The CLI's later stages run in other processes: its prepare must not spend time
    warming kernels for a process that then exits."""
    from cnmf_torch_amd import cli
    from cnmf_torch_amd.api import cNMF

    seen = {}
    monkeypatch.setenv("CNMF_RESIDENT_BYTES", "0")     # (the CLI sets it: restored after)
    monkeypatch.setattr(cNMF, "prepare", lambda self, *a, **kw: seen.update(kw))
    cli.main(["prepare", "-c", str(tmp_path / "none.h5ad"), "-k", "5", "--output-dir",
              str(tmp_path), "--name", "x"])
    assert seen.get("prewarm") is False


@pytest.mark.gpu
def test_prewarm_runs_the_consensus_chain_and_joins():
    dev = torch.device("cuda", 0)
    ts = prewarm.start(dev)
    # one thread (prewarm.start's default) or one per group (prepare's parallel start,
    # when an earlier test of this process ran prepare): started once per process
    assert len(ts) in (1, len(prewarm._GROUPS))
    assert prewarm.start(dev) is ts         # once per process and device
    prewarm.wait(timeout=120)
    assert not any(t.is_alive() for t in ts)
    assert not prewarm.errors, prewarm.errors
    # the warmed stages still compute correctly afterwards
    from cnmf_torch_amd.models.consensus import kmeans

    g = torch.Generator().manual_seed(3)
    X = torch.cat([torch.rand((20, 8), generator=g, dtype=torch.float64) + 4 * i
                   for i in range(3)]).to(dev)
    lab = kmeans(X, 3, backend="device")
    assert len(set(lab[:20])) == 1 and len(set(lab.tolist())) == 3


@pytest.mark.gpu
def test_prepare_builds_the_factorize_planes_ahead(tmp_path, monkeypatch):
    """Opt-in (CNMF_PREBUILD_PLANES=1; off by default since round 6 -- the build is
    factorize's work): prepare (prewarm on) builds the resident matrix's split-GEMM planes
    in the background; factorize in the same process takes them (no second build) and
    factorises bitwise as with a prepare that built nothing ahead."""
    monkeypatch.setenv("CNMF_PREBUILD_PLANES", "1")
    import numpy as np
    import pandas as pd

    from cnmf_torch_amd import cNMF
    from cnmf_torch_amd.models import nmf_base
    from cnmf_torch_amd.utils import resident
    from cnmf_torch_amd.utils.io import load_df_from_npz, save_df_to_npz
    from cnmf_torch_amd.utils.synthetic import simulate_counts

    X, cells, genes = simulate_counts(800, 400, 4, seed=5, sparse=False)
    fn = str(tmp_path / "counts.df.npz")
    save_df_to_npz(pd.DataFrame(X, index=cells, columns=genes), fn)
    spectra = {}
    for warm in (True, False):
        obj = cNMF(output_dir=str(tmp_path / f"w{int(warm)}"), name="p")
        obj.prepare(fn, components=[4], n_iter=3, seed=2, num_highvar_genes=200,
                    prewarm=warm)
        Xr = resident.recall(obj.paths["normalized_counts"], "X32")
        if Xr is None:          # a sparse-stored input: the mirror serves factorize only
            Xr = resident.recall(obj.paths["normalized_counts"], "X32_factorize")
        assert Xr is not None, "prepare kept no device mirror of the normalized counts"
        assert not prewarm.errors, prewarm.errors
        ahead = nmf_base._PLANES_AHEAD.get(Xr)
        assert (ahead is not None) == warm
        calls = []
        orig = nmf_base._XPlanes.__init__

        def counting(self, *a, **kw):
            calls.append(1)
            orig(self, *a, **kw)

        nmf_base._XPlanes.__init__ = counting
        try:
            obj.factorize(verbose=False)
        finally:
            nmf_base._XPlanes.__init__ = orig
        assert len(calls) == (0 if warm else 1)
        spectra[warm] = np.concatenate([
            load_df_from_npz(obj.paths["iter_spectra"] % (4, i)).values for i in range(3)])
    np.testing.assert_array_equal(spectra[True], spectra[False])
