"""N>1 path on the CPU: world_size-2 gloo ranks shard the global problem index,
regenerate their shard, and all-gather (status, iters).  The oracle stands in
for the per-rank solve (CPU-only test of the sharding and the collective)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from socp_amd.dist import shard_range


def test_shard_range_partitions():
    for total in (1, 7, 64, 65536 * 8):
        for world in (1, 2, 3, 8):
            rs = [shard_range(total, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path.insert(0, os.path.join(root, "socp.jl_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch
    import torch.distributed as dist
    import oracle as O
    from socp_amd.configs import C1
    from socp_amd.dist import gather_outcomes, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(total, rank, world)
    cfg = C1
    d = O.generate(cfg.cones, hi - lo, cfg.n, cfg.m, cfg.k, cfg.seed, first_problem=lo)
    r = O.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"],
                      params=O.Params(maxit=40, tol=1e-5), nthreads=1)
    out = gather_outcomes(torch.from_numpy(r["status"]), torch.from_numpy(r["iters"]))
    if rank == 0:
        q.put(out.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_matches_single_process(oracle):
    from socp_amd.configs import C1
    total, world = 16, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cfg = C1
    d = oracle.generate(cfg.cones, total, cfg.n, cfg.m, cfg.k, cfg.seed)
    r = oracle.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"],
                           params=oracle.Params(maxit=40, tol=1e-5), nthreads=1)
    flat = got.reshape(total, 2)
    assert np.array_equal(flat[:, 0], r["status"]) and np.array_equal(flat[:, 1], r["iters"])


@pytest.mark.gpu
def test_abi_status_gather_single_rank():
    """socp_comm_* / socp_allgather_status (the C-ABI RCCL gather a Julia host
    uses) on a one-rank communicator: the output is every rank's interleaved
    (status, iters).  More ranks need more GPUs than a test box has; the
    torch.distributed path of bench.py covers N > 1."""
    import torch
    import socp_amd as S
    from socp_amd.dist import StatusComm
    ctx = S.default_context()
    uid = StatusComm.unique_id()
    assert len(uid) == 128
    comm = StatusComm(ctx, 1, 0, uid)
    try:
        B = 1000
        st = torch.randint(0, 5, (B,), dtype=torch.int32, device="cuda")
        it = torch.randint(0, 41, (B,), dtype=torch.int32, device="cuda")
        out = comm.allgather_status(st, it)
        assert out.shape == (1, B, 2)
        assert torch.equal(out[0, :, 0], st) and torch.equal(out[0, :, 1], it)
    finally:
        comm.close()
