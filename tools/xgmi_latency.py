"""Per-call time of the one-shot xGMI collectives (parallel/xgmi.py) with 2 processes on
ONE GPU: the flag handshake, staging and peer reads run as across the GPUs of a node, so
the small-message time is the kernels' per-call latency (the fixed term of the DP
projection in tools/bench_large.py --emulate-world); the peer reads here stay on one
GPU's HBM, so the bandwidth term is modelled separately (bytes / xGMI link bandwidth).

    python tools/xgmi_latency.py > profiles/r5_xgmi_latency.json
"""
import json
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

SIZES = [1 << 10, 1 << 16, 1 << 20, 1 << 22]      # float32 elements of the full buffer
CALLS = 200


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from cnmf_torch_amd.parallel.xgmi import XgmiAllReduce

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    xg = XgmiAllReduce(None, dev, cap=max(SIZES), timeout_ms=5000)
    out = {}
    for n in SIZES:
        m = n // world
        a = torch.randn(n, device=dev)
        o = torch.empty(m, device=dev)
        b = torch.randn(m, device=dev)
        ob = torch.empty(n, device=dev)
        for name, fn in (("all_reduce", lambda: xg(a)),
                         ("reduce_scatter", lambda: xg.reduce_scatter(o, a)),
                         ("all_gather", lambda: xg.all_gather(ob, b))):
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(CALLS):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / CALLS
            out[f"{name}_{n * 4}B_us"] = round(dt * 1e6, 2)
    xg.check()
    xg.close()
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
    small = [v for k, v in res.items() if k.endswith(f"_{SIZES[0] * 4}B_us")]
    print(json.dumps({"metric": "one-shot xGMI collective time per call, 2 ranks on one GPU",
                      "unit": "us", "per_call_us": res,
                      "latency_us": round(max(small), 2),
                      "note": "latency_us = the slowest kind at 4 KB (fixed per-call term)",
                      "device": torch.cuda.get_device_name(0)}))


if __name__ == "__main__":
    main()
