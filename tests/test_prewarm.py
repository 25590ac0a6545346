"""utils.prewarm: the background first-use loading cNMF.prepare starts on a GPU."""
import pytest
import torch

from cnmf_torch_amd.utils import prewarm


def test_prewarm_is_a_noop_off_the_gpu():
    assert prewarm.start("cpu") is None
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
    t = prewarm.start(dev)
    assert t is not None
    assert prewarm.start(dev) is t          # once per process and device
    prewarm.wait(timeout=120)
    assert not t.is_alive()
    # the warmed stages still compute correctly afterwards
    from cnmf_torch_amd.models.consensus import kmeans

    g = torch.Generator().manual_seed(3)
    X = torch.cat([torch.rand((20, 8), generator=g, dtype=torch.float64) + 4 * i
                   for i in range(3)]).to(dev)
    lab = kmeans(X, 3, backend="device")
    assert len(set(lab[:20])) == 1 and len(set(lab.tolist())) == 3
