"""N>1 path on the CPU: world_size-2 gloo ranks shard the global problem index,
regenerate their shard, and all-gather the 32-byte outcome records (status,
iters, ||rd||, ||rp||, z's: SURVEY.md §8(e)).  The oracle stands in for the
per-rank solve (CPU-only test of the sharding and the collective)."""
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
    out = gather_outcomes(torch.from_numpy(r["status"]), torch.from_numpy(r["iters"]),
                          torch.from_numpy(r["res"]))
    if rank == 0:
        q.put({key: v.numpy() for key, v in out.items()})
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
    assert got["status"].shape == (world, total // world)
    assert np.array_equal(got["status"].reshape(-1), r["status"])
    assert np.array_equal(got["iters"].reshape(-1), r["iters"])
    # residual norms travel bit-exactly (the oracle is deterministic per problem)
    assert np.array_equal(got["res"].reshape(total, 3), r["res"])


def test_outcome_record_layout():
    """pack/unpack of the socp_outcome record (include/socp.h): 32 bytes, int32
    status and iters first, then three float64."""
    import torch
    from socp_amd.dist import RECORD_BYTES, pack_outcomes, unpack_outcomes
    st = torch.tensor([0, 1, 4], dtype=torch.int32)
    it = torch.tensor([7, 40, 3], dtype=torch.int32)
    res = torch.tensor([[1e-6, 2e-7, 3e-8], [1.5, 2.5, 3.5], [float("inf"), -0.0, 5.0]], dtype=torch.float64)
    rec = pack_outcomes(st, it, res)
    assert rec.shape == (3, RECORD_BYTES) and RECORD_BYTES == 32
    raw = rec.numpy().tobytes()
    import struct
    for p in range(3):
        s_, i_, a, b, c = struct.unpack_from("<iiddd", raw, 32 * p)
        assert (s_, i_) == (int(st[p]), int(it[p]))
        assert [a, b, c] == res[p].tolist()
    back = unpack_outcomes(rec)
    assert torch.equal(back["status"], st) and torch.equal(back["iters"], it)
    assert torch.equal(back["res"], res)
    nan = unpack_outcomes(pack_outcomes(st, it))["res"]
    assert torch.isnan(nan).all()


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
        # the 32-byte record with the residual norms of a real solve
        from socp_amd.configs import C1
        cfg = C1
        c, A, b, G, h = S.generate(cfg.cones, 64, cfg.n, cfg.m, cfg.k, cfg.seed, ctx=ctx)
        o = S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, c, A, b, G, h,
                          torch.zeros(64, dtype=torch.uint8, device="cuda"), maxit=40, tol=1e-5, ctx=ctx,
                          res=True)
        rec = comm.allgather_outcomes(o["status"], o["iters"], o["res"])
        assert rec["status"].shape == (1, 64)
        assert torch.equal(rec["status"][0], o["status"]) and torch.equal(rec["iters"][0], o["iters"])
        assert torch.equal(rec["res"][0], o["res"].view(64, 3))
        conv = o["status"] == 0
        assert conv.any()
        # converged problems satisfy the reference exit test (solver.jl:122)
        assert (rec["res"][0][conv].sum(dim=1) < 1e-5).all()
    finally:
        comm.close()
