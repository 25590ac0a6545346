"""Worker entry points for multi-process tests (spawned with torch.multiprocessing)."""
import os

import numpy as np
import torch
import torch.distributed as dist


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    os.environ["LOCAL_RANK"] = str(rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)


def dp_solver_worker(rank, world, port, X, K, seeds, opts_kw, out_dir):
    _init(rank, world, port)
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions
    from cnmf_torch_amd.parallel.comm import DistComm
    from cnmf_torch_amd.parallel.runner import dp_layout, dp_row_segments

    segs = dp_row_segments(X.shape[0], opts_kw["online_chunk_size"], rank, world)
    row_map, sched = dp_layout(segs)
    Xl = torch.from_numpy(np.concatenate([X[a:b] for a, b in segs]))
    solver = NMFBatchSolver(Xl, NMFOptions(n_components=K, **opts_kw), comm=DistComm(),
                            row_map=row_map, schedule=sched)
    res = solver.run(seeds, ks=opts_kw.get("_ks"))
    np.save(os.path.join(out_dir, f"rows{rank}.npy"),
            np.concatenate([np.arange(a, b) for a, b in segs]))
    np.save(os.path.join(out_dir, f"W{rank}.npy"), res.W.numpy())
    np.save(os.path.join(out_dir, f"HT{rank}.npy"), res.HT.numpy())
    np.save(os.path.join(out_dir, f"err{rank}.npy"), res.err)
    dist.barrier()
    dist.destroy_process_group()


def factorize_worker(rank, world, port, output_dir, name, mode):
    _init(rank, world, port)
    from cnmf_torch_amd import cNMF
    from cnmf_torch_amd.parallel.runner import distributed_factorize, dp_factorize

    obj = cNMF(output_dir=output_dir, name=name)
    if mode == "replicate":
        distributed_factorize(obj, backend="gloo", verbose=False)
    elif mode == "gather":      # resume + gather: completed replicates come from files
        distributed_factorize(obj, backend="gloo", verbose=False, gather_spectra=True,
                              skip_completed_runs=True)
    else:
        dp_factorize(obj, backend="gloo", verbose=False)
    dist.destroy_process_group()


def comm_worker(rank, world, port, out_dir):
    _init(rank, world, port)
    from cnmf_torch_amd.parallel.comm import DistComm

    c = DistComm()
    t = torch.full((5,), float(rank + 1))
    c.allreduce_(t)
    s = c.allreduce_scalar(rank + 0.5)
    m = c.allreduce_max_int(rank * 10)
    g = c.all_gather_object({"r": rank})
    # the background forms: both issued before either is waited on
    o = torch.empty(2)
    ob = torch.empty(3 * world, dtype=torch.int16)
    h1 = c.reduce_scatter_async(o, torch.arange(2 * world, dtype=torch.float32) + rank)
    h2 = c.all_gather_into_async(ob, torch.full((3,), rank + 7, dtype=torch.int16))
    h1.wait()
    h2.wait()
    exp_o = sum(torch.arange(2 * world, dtype=torch.float32) + r for r in range(world))
    ok = bool(torch.equal(o, exp_o[2 * rank:2 * rank + 2])) and \
        bool(torch.equal(ob, torch.arange(world, dtype=torch.int16).repeat_interleave(3) + 7))
    np.save(os.path.join(out_dir, f"comm{rank}.npy"),
            np.array([t[0].item(), s, m, len(g), g[world - 1]["r"], float(ok)]))
    dist.destroy_process_group()


def fault_worker(rank, world, port, output_dir, name, fault_rank):
    """Replicate-parallel factorize where ``fault_rank`` dies after one replicate
    (CNMF_FAULT_AFTER_REPLICATES); every rank records how it ended and exits."""
    import datetime

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    if rank == fault_rank:
        os.environ["CNMF_FAULT_AFTER_REPLICATES"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=30))
    torch.set_num_threads(1)
    from cnmf_torch_amd import cNMF
    from cnmf_torch_amd.parallel.runner import distributed_factorize

    status = "ok"
    try:
        distributed_factorize(cNMF(output_dir=output_dir, name=name), backend="gloo",
                              verbose=False)
    except Exception as e:  # the injected fault, or the peer's disappearance
        status = type(e).__name__ + ": " + str(e)[:200]
    with open(os.path.join(output_dir, f"status{rank}.txt"), "w") as fh:
        fh.write(status)
    os._exit(0)


def resume_worker(rank, world, port, output_dir, name):
    _init(rank, world, port)
    from cnmf_torch_amd import cNMF
    from cnmf_torch_amd.parallel.runner import distributed_factorize

    distributed_factorize(cNMF(output_dir=output_dir, name=name), skip_completed_runs=True,
                          backend="gloo", verbose=False)
    dist.destroy_process_group()


def consensus_worker(rank, world, port, output_dir, name, ks):
    _init(rank, world, port)
    from cnmf_torch_amd import cNMF
    from cnmf_torch_amd.parallel.runner import distributed_consensus, distributed_k_selection

    obj = cNMF(output_dir=output_dir, name=name)
    distributed_k_selection(obj, backend="gloo")
    distributed_consensus(obj, ks, density_threshold=0.5, show_clustering=False,
                          backend="gloo")
    dist.destroy_process_group()


def prepare_worker(rank, world, port, output_dir, name, counts_fn, kw):
    _init(rank, world, port)
    from cnmf_torch_amd import cNMF
    from cnmf_torch_amd.parallel.comm import DistComm

    os.environ["CNMF_PREPARE_CHUNK_BYTES"] = str(kw.pop("_chunk_bytes", 1 << 30))
    from cnmf_torch_amd.models import hvg

    comm = DistComm()
    cNMF(output_dir=output_dir, name=name).prepare(counts_fn, comm=comm, **kw)
    np.save(os.path.join(output_dir, f"maxmsg{rank}.npy"), np.array([comm.max_msg_bytes]))
    np.save(os.path.join(output_dir, f"devblocks{rank}.npy"),
            np.array([hvg.DEVICE_MOMENT_BLOCKS]))
    dist.destroy_process_group()


def tp_consensus_worker(rank, world, port, output_dir, name, k):
    _init(rank, world, port)
    from cnmf_torch_amd import cNMF
    from cnmf_torch_amd.parallel.runner import distributed_consensus

    distributed_consensus(cNMF(output_dir=output_dir, name=name), [k], density_threshold=0.5,
                          show_clustering=False, backend="gloo")
    dist.destroy_process_group()


def xgmi_worker(rank, world, port, out_dir):
    """One-shot xGMI all-reduce against gloo's (several processes on ONE GPU here: the IPC
    mapping and the flag handshake are the same as across the GPUs of a node)."""
    _init(rank, world, port)
    from cnmf_torch_amd.parallel.comm import DistComm
    from cnmf_torch_amd.parallel.xgmi import XgmiAllReduce, XgmiTimeout

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    xg = XgmiAllReduce(None, dev, cap=1 << 16, timeout_ms=3000)
    res = {"memory_kind": xg.memory_kind}
    # back-to-back calls without host syncs (both workspace parities in flight); sizes hit
    # the float4 body, scalar tails and a buffer at capacity; an unaligned view too
    sizes = [1, 3, 4, 1000, 4097, 1 << 16, 777, 65533, 5, 4096] * 6
    ins, outs = [], []
    for i, n in enumerate(sizes):
        g = torch.Generator().manual_seed(1000 * i + rank)
        t = torch.randn(n, generator=g).to(dev)
        ins.append(t.cpu())
        if i % 3 == 2:      # out of place
            o = torch.empty_like(t)
            outs.append(xg(t, o))
        else:
            outs.append(xg(t))
    unal = torch.randn(1 << 12 | 1, generator=torch.Generator().manual_seed(rank)).to(dev)[1:]
    ins.append(unal.cpu())
    outs.append(xg(unal))
    torch.cuda.synchronize()
    xg.check()
    for i, (a, o) in enumerate(zip(ins, outs)):
        ref = a.clone()
        dist.all_reduce(ref)
        res[f"err{i}"] = float((o.cpu() - ref).abs().max())
        res[f"sum{i}"] = o.cpu().numpy()
    # DistComm routes device float32 buffers here under CNMF_ALLREDUCE=xgmi
    os.environ["CNMF_ALLREDUCE"] = "xgmi"
    comm = DistComm()
    t = torch.full((10,), float(rank + 1), device=dev)
    comm.allreduce_(t)
    comm.check()
    res["comm"] = t.cpu().numpy()
    res["comm_is_xgmi"] = bool(comm._xgmi)
    comm.close()
    # a rank that never arrives: the kernel gives up after the limit, and the (collective)
    # check raises on EVERY rank, the one that waited and the one that never came
    timed_out = False
    dist.barrier()
    xg.limit = xg.limit // 3000 * 200                       # 200 ms
    if rank == 0:
        xg(torch.ones(64, device=dev))
        torch.cuda.synchronize()
    try:
        xg.check()
    except XgmiTimeout:
        timed_out = True
    res["timed_out"] = timed_out
    xg.close()
    np.savez(os.path.join(out_dir, f"xgmi{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


def xgmi_dp_worker(rank, world, port, X, K, seeds, opts_kw, out_dir, allreduce):
    """Cell-sharded DP solve on one GPU per process with the all-reduce over xGMI peer
    memory or staged through gloo."""
    os.environ["CNMF_ALLREDUCE"] = allreduce
    os.environ["CNMF_DP_FUSED"] = "0"     # the all-reduced step (the fused one reduce-scatters)
    # both ranks share one GPU here: no cooperative (co-residency assuming) solves
    os.environ["CNMF_SOLVE_COOP"] = "0"
    _init(rank, world, port)
    from cnmf_torch_amd import ops
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions

    ops.refresh_env()
    from cnmf_torch_amd.parallel.comm import DistComm
    from cnmf_torch_amd.parallel.runner import dp_layout, dp_row_segments

    torch.cuda.set_device(0)
    segs = dp_row_segments(X.shape[0], opts_kw["online_chunk_size"], rank, world)
    row_map, sched = dp_layout(segs)
    Xl = torch.from_numpy(np.concatenate([X[a:b] for a, b in segs])).cuda()
    comm = DistComm()
    solver = NMFBatchSolver(Xl, NMFOptions(n_components=K, **opts_kw), comm=comm,
                            row_map=row_map, schedule=sched)
    res = solver.run(seeds)
    np.save(os.path.join(out_dir, f"W_{allreduce}{rank}.npy"), res.W.cpu().numpy())
    np.save(os.path.join(out_dir, f"err_{allreduce}{rank}.npy"), res.err)
    res_xg = bool(comm._xgmi)
    np.save(os.path.join(out_dir, f"used_{allreduce}{rank}.npy"), np.array(res_xg))
    comm.close()
    dist.barrier()
    dist.destroy_process_group()


def xgmi_rsag_worker(rank, world, port, out_dir):
    """One-shot xGMI reduce-scatter / all-gather (and all-reduce between them, one device
    call counter for all three) against gloo, eagerly and replayed from a HIP graph."""
    _init(rank, world, port)
    from cnmf_torch_amd.parallel.comm import DistComm
    from cnmf_torch_amd.parallel.xgmi import XgmiAllReduce

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    xg = XgmiAllReduce(None, dev, cap=1 << 16, timeout_ms=3000)
    res = {}
    k = 0

    def rs_ref(inp):
        h = inp.cpu().clone()
        dist.all_reduce(h)
        m = h.numel() // world
        return h[rank * m:(rank + 1) * m]

    def ag_ref(inp):          # (gloo has no int16 all-gather: as bytes)
        h = inp.cpu().contiguous().view(torch.uint8)
        parts = [torch.empty_like(h) for _ in range(world)]
        dist.all_gather(parts, h)
        return torch.cat(parts).view(inp.dtype)

    for i, m in enumerate([5, 1000, 4096, 777, 8, 4097] * 2):
        g = torch.Generator().manual_seed(100 * i + rank)
        a = torch.randn(world * m, generator=g).to(dev)
        o = torch.empty(m, device=dev)
        assert xg.reduce_scatter(o, a)
        b = torch.randn(m, generator=g).to(dev)
        ob = torch.empty(world * m, device=dev)
        assert xg.all_gather(ob, b)
        c = torch.randint(-30000, 30000, (2 * m,), generator=g, dtype=torch.int16).to(dev)
        oc = torch.empty(world * 2 * m, dtype=torch.int16, device=dev)
        assert xg.all_gather(oc, c)
        d = torch.randn(m, generator=g).to(dev)
        dd = d.clone()
        xg(dd)
        torch.cuda.synchronize()
        res[f"rs{k}"] = float((o.cpu() - rs_ref(a)).abs().max())
        res[f"ag{k}"] = float((ob.cpu() - ag_ref(b)).abs().max())
        res[f"agi{k}"] = int((oc.cpu() != ag_ref(c)).sum())
        dref = d.cpu().clone()
        dist.all_reduce(dref)
        res[f"ar{k}"] = float((dd.cpu() - dref).abs().max())
        k += 1
    # the same calls captured once and replayed with new inputs: the device call counter
    # advances on every replay
    m = 1000
    a = torch.zeros(world * m, device=dev)
    o = torch.empty(m, device=dev)
    b = torch.zeros(m, device=dev)
    ob = torch.empty(world * m, device=dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            xg.reduce_scatter(o, a)
            xg.all_gather(ob, b)
    torch.cuda.current_stream(dev).wait_stream(s)
    for r_ in range(3):
        g = torch.Generator().manual_seed(7000 + 10 * r_ + rank)
        a.copy_(torch.randn(world * m, generator=g))
        b.copy_(torch.randn(m, generator=g))
        graph.replay()
        torch.cuda.synchronize()
        res[f"grs{r_}"] = float((o.cpu() - rs_ref(a)).abs().max())
        res[f"gag{r_}"] = float((ob.cpu() - ag_ref(b)).abs().max())
    xg.check()
    res["n"] = k
    xg.close()
    # DistComm routes reduce-scatter / all-gather here under CNMF_ALLREDUCE=xgmi
    os.environ["CNMF_ALLREDUCE"] = "xgmi"
    comm = DistComm()
    o = torch.empty(3, device=dev)
    comm.reduce_scatter_(o, torch.full((3 * world,), float(rank + 1), device=dev))
    ob = torch.empty(4 * world, dtype=torch.int16, device=dev)
    comm.all_gather_into_(ob, torch.full((4,), rank + 7, dtype=torch.int16, device=dev))
    # two exchanges in flight on the side stream while the current stream computes
    o2 = torch.empty(5, device=dev)
    ob2 = torch.empty(6 * world, dtype=torch.int16, device=dev)
    h1 = comm.reduce_scatter_async(o2, torch.full((5 * world,), 2.0 * (rank + 1), device=dev))
    busy = torch.randn(2048, 2048, device=dev)
    busy = busy @ busy
    h2 = comm.all_gather_into_async(ob2, torch.full((6,), rank + 3, dtype=torch.int16,
                                                    device=dev))
    h1.wait()
    h2.wait()
    comm.check()
    res["comm_rs"] = o.cpu().numpy()
    res["comm_ag"] = ob.cpu().numpy()
    res["comm_rs_async"] = o2.cpu().numpy()
    res["comm_ag_async"] = ob2.cpu().numpy()
    res["comm_is_xgmi"] = bool(comm._xgmi)
    comm.close()
    np.savez(os.path.join(out_dir, f"rsag{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


def dp_fused_worker(rank, world, port, X, K, seeds, opts_kw, out_dir, fused, allreduce="rccl"):
    """Cell-sharded DP solve on the GPU (both ranks share the one GPU of the box; the
    collectives are staged through gloo, or -- allreduce="xgmi" -- run as the one-shot
    peer-memory kernels): the packed reduce-scatter / all-gather fused step
    (CNMF_DP_FUSED=1) or the all-reduced unfused step (0)."""
    os.environ["CNMF_DP_FUSED"] = fused
    os.environ["CNMF_ALLREDUCE"] = allreduce
    # the production cooperative-slice solves (S_h, S_w > 1): both processes share one
    # GPU here, and a launch of these sizes is a few dozen workgroups -- every slice of
    # both ranks' launches is resident at once
    os.environ.pop("CNMF_SOLVE_COOP", None)
    _init(rank, world, port)
    from cnmf_torch_amd import ops
    from cnmf_torch_amd.models.nmf import NMFBatchSolver, NMFOptions, _Batch

    ops.refresh_env()
    from cnmf_torch_amd.parallel.comm import DistComm
    from cnmf_torch_amd.parallel.runner import dp_layout, dp_row_segments

    torch.cuda.set_device(0)
    segs = dp_row_segments(X.shape[0], opts_kw["online_chunk_size"], rank, world)
    row_map, sched = dp_layout(segs)
    Xl = torch.from_numpy(np.concatenate([X[a:b] for a, b in segs])).cuda()
    ks = list(K) if isinstance(K, (list, tuple)) else [K] * len(seeds)   # mixed-K batch
    solver = NMFBatchSolver(Xl, NMFOptions(n_components=ks[0], **opts_kw), comm=DistComm(),
                            row_map=row_map, schedule=sched)
    st = _Batch(torch.zeros((sum(ks), Xl.shape[0]), device="cuda"),
                torch.zeros((sum(ks), Xl.shape[1]), device="cuda"), sorted(ks))
    took = solver._fused_ok(st, solver._steps(Xl.shape[0]))
    res = solver.run(seeds, ks=ks)
    tag = fused + ("x" if allreduce == "xgmi" else "")
    np.save(os.path.join(out_dir, f"dpf{tag}_{rank}.npz.npy"),
            np.array([took, bool(solver.comm._xgmi)], dtype=bool))
    np.save(os.path.join(out_dir, f"dpfS{tag}_{rank}.npy"),
            np.array(tuple(getattr(solver, "dp_slices", (0, 0)))
                     + (getattr(solver, "dp_units", 0),), dtype=np.int64))
    np.save(os.path.join(out_dir, f"dpfW{tag}_{rank}.npy"), res.W.cpu().numpy())
    np.save(os.path.join(out_dir, f"dpferr{tag}_{rank}.npy"), res.err)
    np.save(os.path.join(out_dir, f"dpfit{tag}_{rank}.npy"), res.n_iter)
    solver.comm.close()
    dist.barrier()
    dist.destroy_process_group()
