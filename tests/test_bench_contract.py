"""bench.py contract: one JSON line from rank 0, whole-job value, max-over-ranks timing.
Runs the multi-rank path on the CPU (gloo, 2 and 8 ranks via torch.distributed.run) --
8 is the driver's scaling world."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(extra, nproc):
    tiny = ["--cpu", "--cells", "300", "--genes", "60", "--k", "4", "--n-iter", "3",
            "--batch-size", "100", "--max-nmf-iter", "50", "--steps", "2", "--warmup", "1"]
    if nproc == 1:
        cmd = [sys.executable, "bench.py"] + tiny + extra
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={nproc}", "--master-addr", "127.0.0.1", "--master-port",
               str(_port()), "bench.py", "--gpus", str(nproc)] + tiny + extra
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    return json.loads(lines[0])


def test_bench_json_contract_two_ranks():
    out = _bench([], 2)
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in out, key
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["scaling"] == "weak" and out["higher_is_better"] is True
    assert out["config"]["global_batch"] == 6            # 3 replicates per rank
    # value is the whole-job rate: global replicates * steps / (max-rank) elapsed
    rate = 6 * 2 / (out["ms_per_step"] * 2 / 1000.0)
    assert abs(out["value"] - rate) / out["value"] < 0.01


def test_bench_strong_and_dp_modes_two_ranks():
    strong = _bench(["--mode", "strong"], 2)
    assert strong["scaling"] == "strong" and strong["config"]["global_batch"] == 3
    dp = _bench(["--mode", "dp"], 2)
    assert dp["scaling"] == "strong" and dp["config"]["global_batch"] == 3
    assert dp["config"]["parallelism"].startswith("cell-sharded DP x2")
    assert "RCCL" in dp["config"]["parallelism"]
    rate = 3 * 2 / (dp["ms_per_step"] * 2 / 1000.0)
    assert abs(dp["value"] - rate) / dp["value"] < 0.01
    # the xGMI option only reroutes device buffers: the CPU (gloo) run is unchanged
    xg = _bench(["--mode", "dp", "--allreduce", "xgmi"], 2)
    assert "one-shot xGMI" in xg["config"]["parallelism"]
    assert xg["config"]["mean_passes"] == dp["config"]["mean_passes"]


def test_bench_dp_mode_same_factorisation_as_one_rank():
    """The DP bench solves the same replicates as the one-GPU bench: same mean passes."""
    one = _bench(["--mode", "dp"], 1)
    two = _bench(["--mode", "dp"], 2)
    assert abs(one["config"]["mean_passes"] - two["config"]["mean_passes"]) <= 0.5


def test_bench_k_grid_ragged_batch():
    out = _bench(["--kmin", "3", "--kmax", "5"], 1)
    assert out["config"]["global_batch"] == 9 and out["metric"].startswith(
        "NMF replicates/sec (K=3..5")


def test_bench_self_launches_n_ranks_without_a_launcher():
    """``python bench.py --gpus 2`` with no torch.distributed.run in front starts the two
    ranks itself (child launcher, never an exec) and reports the process-group world."""
    tiny = ["--cpu", "--cells", "300", "--genes", "60", "--k", "4", "--n-iter", "3",
            "--batch-size", "100", "--max-nmf-iter", "50", "--steps", "2", "--warmup", "1"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"] + tiny, cwd=ROOT,
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["rccl_world"] == 2
    assert out["config"]["backend"] == "gloo"
    # weak run also reports the strong form: one 3-replicate batch per step over 2 ranks
    assert out["config"]["strong_global_batch"] == 3
    assert out["config"]["strong_value"] > 0


def test_bench_world_size_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0",
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "bench.py", "--cpu", "--gpus", "2"], cwd=ROOT,
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_eight_ranks_weak_strong_dp():
    """The driver's N=8 launch shape on gloo: weak (3 replicates per rank, 24 per step),
    strong (ONE 3-replicate ledger batch over 8 ranks: five ranks own nothing) and dp
    (300 cells in 100-cell chunks over 8 ranks: 12-13 cells per rank and chunk) all
    complete and print one whole-job JSON line; weak reports its strong form too."""
    weak = _bench([], 8)
    assert weak["n_gpus"] == 8 and weak["config"]["rccl_world"] == 8
    assert weak["config"]["global_batch"] == 24 and weak["scaling"] == "weak"
    assert weak["config"]["strong_value"] > 0 and weak["config"]["strong_global_batch"] == 3
    rate = 24 * 2 / (weak["ms_per_step"] * 2 / 1000.0)
    assert abs(weak["value"] - rate) / weak["value"] < 0.01
    strong = _bench(["--mode", "strong"], 8)
    assert strong["config"]["global_batch"] == 3 and strong["scaling"] == "strong"
    dp = _bench(["--mode", "dp"], 8)
    assert dp["config"]["parallelism"].startswith("cell-sharded DP x8")
    one = _bench(["--mode", "dp"], 1)
    assert abs(one["config"]["mean_passes"] - dp["config"]["mean_passes"]) <= 0.5
