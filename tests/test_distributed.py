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


def _bench_worker(rank, world, port, total, steps, q):
    """One rank of bench.py's N>1 loop (socp_amd.dist.timed_shard_steps) over
    gloo, with the oracle as the per-rank shard solve."""
    import sys
    import time
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path.insert(0, os.path.join(root, "socp.jl_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch
    import torch.distributed as dist
    import oracle as O
    from socp_amd.configs import C1
    from socp_amd.dist import shard_range, timed_shard_steps
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(total, rank, world)
    cfg = C1
    d = O.generate(cfg.cones, hi - lo, cfg.n, cfg.m, cfg.k, cfg.seed, first_problem=lo)
    calls = []

    def solve_shard():
        if rank == 1:
            time.sleep(0.05)  # a slower rank: the reported time must be the max
        r = O.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"],
                          params=O.Params(maxit=40, tol=1e-5), nthreads=1)
        calls.append(1)
        return {key: torch.from_numpy(r[key]) for key in ("status", "iters", "res")}

    tr = timed_shard_steps(solve_shard, steps, 1)
    q.put({"rank": rank, "dt": tr["dt"], "iters_total": tr["iters_total"], "iters_local": tr["iters_local"],
           "calls": len(calls), "step_ms": tr["step_ms"],
           "gathered": {key: v.numpy() for key, v in tr["gathered"].items()}})
    dist.barrier()
    dist.destroy_process_group()


def test_bench_step_accounting_gloo_world2(oracle):
    """bench.py's N>1 accounting on the CPU: two gloo ranks run the timed step
    loop; the iteration total, the max-over-ranks time and the gathered
    records equal what a single process computes for the whole batch."""
    from socp_amd.configs import C1
    total, world, steps = 8, 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, total, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=180) for _ in range(world)], key=lambda g: g["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cfg = C1
    d = oracle.generate(cfg.cones, total, cfg.n, cfg.m, cfg.k, cfg.seed)
    r = oracle.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"],
                           params=oracle.Params(maxit=40, tol=1e-5), nthreads=1)
    single_iters = int(r["iters"].sum()) * steps
    for g in got:
        assert g["calls"] == steps + 1  # one warm-up step, then exactly `steps`
        assert g["iters_total"] == single_iters
        assert np.array_equal(g["gathered"]["status"].reshape(-1), r["status"])
        assert np.array_equal(g["gathered"]["iters"].reshape(-1), r["iters"])
        assert np.array_equal(g["gathered"]["res"].reshape(total, 3), r["res"])
    assert got[0]["iters_local"] + got[1]["iters_local"] == single_iters
    # every rank reports the same, max-over-ranks time, at least the slow rank's own steps
    assert got[0]["dt"] == got[1]["dt"]
    assert got[0]["dt"] >= sum(got[1]["step_ms"]) / 1e3 - 1e-6
    assert got[0]["dt"] >= steps * 0.05


@pytest.mark.gpu
def test_abi_outcome_gather_fresh_context_converted_inputs():
    """socp_allgather_outcomes on a fresh Context whose stream nothing has bound
    yet, with int64 status / iters and float32 residuals: the conversions run
    on torch's stream and the gather must see them (StatusComm binds the
    context to torch's stream first)."""
    import torch
    import socp_amd as S
    from socp_amd.dist import StatusComm
    ctx = S.Context(0)
    comm = StatusComm(ctx, 1, 0, StatusComm.unique_id())
    try:
        for B in (1, 4097, 200000):
            st = torch.randint(0, 5, (B,), dtype=torch.int64, device="cuda")
            it = torch.randint(0, 41, (B,), dtype=torch.int64, device="cuda")
            res = torch.rand((B, 3), dtype=torch.float32, device="cuda") * 1e-3
            rec = comm.allgather_outcomes(st, it, res)
            assert torch.equal(rec["status"][0], st.to(torch.int32))
            assert torch.equal(rec["iters"][0], it.to(torch.int32))
            assert torch.equal(rec["res"][0], res.to(torch.float64))
            out = comm.allgather_status(st, it)
            assert torch.equal(out[0, :, 0], st.to(torch.int32)) and torch.equal(out[0, :, 1], it.to(torch.int32))
    finally:
        comm.close()


def _bench_env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env["CUDA_VISIBLE_DEVICES"] = ""  # the stub ranks never touch a GPU
    env["OMP_NUM_THREADS"] = "1"
    return env


def _bench_json(stdout):
    import json
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_bench_launcher_starts_n_ranks():
    """`python bench.py --gpus 2` with no launcher starts two ranks itself
    (torch.distributed.run from a parent that never touches the GPU); rank 0
    prints one line for the whole job: n_gpus 2, global batch 2 B, the
    iterations of both shards over the max-over-ranks time.  The shard solve
    is bench.py's --stub-solve (gloo, K iterations per problem, no GPU)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    B, steps, K = 96, 3, 8
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", str(steps),
                        "--warmup", "1", "--batch", str(B), "--stub-solve"],
                       capture_output=True, text=True, timeout=300, env=_bench_env(), cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _bench_json(r.stdout)
    assert line["n_gpus"] == 2
    assert line["config"]["global_batch"] == 2 * B
    assert line["config"]["parallelism"].startswith("dp2")
    assert line["steps"] == steps and line["warmup"] == 1
    # value = every rank's problem-iterations / the max-over-ranks time of the timed steps
    dt = line["ms_per_step"] * steps / 1e3
    assert abs(line["value"] * dt - 2 * B * K * steps) <= 1e-6 * 2 * B * K * steps
    assert line["ms_per_step"] >= 10.0  # the stub's 10 ms per step
    assert line["cpu_baseline"] is None  # the CPU leg runs at N=1 only
    # rank 0 holds every rank's outcome records after the exchange step
    assert line["gathered"] == {"status_counts": [2 * B, 0, 0, 0, 0], "iters_sum": 2 * B * K, "problems": 2 * B}


@pytest.mark.gpu
def test_bench_two_ranks_real_solves_on_one_gpu():
    """The N > 1 path end to end with the HIP solver on the one-GPU box:
    `bench.py --gpus 2 --dist-backend gloo` starts two ranks (sharing the GPU;
    the line is marked a rehearsal), each generates and solves its own shard
    (problems rank * B ... of the generator's sequence) under the reference
    stopping rule, and rank 0 gathers every 32-byte outcome record.  The
    gathered outcomes must be those of one rank solving all 2 B problems:
    the same status histogram and the same total iteration count (each
    problem is solved independently, so sharding changes nothing)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    B = 2048
    common = ["--mode", "reference", "--steps", "1", "--warmup", "0", "--no-cpu", "--no-ingest"]
    two = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                          "--batch", str(B)] + common, capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert two.returncode == 0, two.stderr[-3000:]
    one = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--batch", str(2 * B)] + common,
                         capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert one.returncode == 0, one.stderr[-3000:]
    l2, l1 = _bench_json(two.stdout), _bench_json(one.stdout)
    assert l2["n_gpus"] == 2 and l2["config"]["global_batch"] == 2 * B
    assert "REHEARSAL" in l2["config"]["parallelism"]
    assert l2["gathered"]["problems"] == 2 * B
    assert l2["gathered"]["status_counts"] == l1["status_counts"], (l2["gathered"], l1["status_counts"])
    assert l2["gathered"]["iters_sum"] == l1["roofline"]["problem_iters_per_launch"]
    assert sum(l2["status_counts"]) == B  # rank 0's own shard


def test_bench_one_gpu_line_unchanged_shape():
    """--gpus 1 stays one process: n_gpus 1, global batch B."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--batch", "32", "--stub-solve", "--no-cpu"],
                       capture_output=True, text=True, timeout=300, env=_bench_env(), cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _bench_json(r.stdout)
    assert line["n_gpus"] == 1 and line["config"]["global_batch"] == 32
    assert line["config"]["parallelism"].startswith("dp1")


def test_bench_line_carries_the_driver_contract():
    """The one JSON line keeps every key the driver and the judge read: the
    metric / value / unit / n_gpus / steps / warmup / ms_per_step block, the
    config naming the workload, roofline (bound, achieved, peak, unit, frac,
    traffic) and cpu_baseline (null at --no-cpu).  Stub solve, CPU only."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--batch", "32", "--stub-solve", "--no-cpu"],
                       capture_output=True, text=True, timeout=300, env=_bench_env(), cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _bench_json(r.stdout)
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in line, key
    assert line["unit"] == "problem-iterations/s" and line["higher_is_better"] is True
    assert line["scaling"] == "weak" and line["dtype"] == "f64" and line["vs_baseline"] is None
    assert line["steps"] == 2 and line["warmup"] == 1 and line["n_gpus"] == 1
    assert {"workload", "global_batch", "parallelism"} <= set(line["config"])
    roof = line["roofline"]
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(roof)
    assert roof["bound"] in ("hbm", "mfma") and roof["unit"] in ("GB/s", "TFLOP/s")
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) <= 1e-12 * max(1.0, roof["frac"])
    assert line["cpu_baseline"] is None


def test_bench_world_size_mismatch_fails():
    """Under a launcher, WORLD_SIZE must equal --gpus: a mismatch exits non-zero
    before any process group or device is touched."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = _bench_env()
    env.update(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--stub-solve"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=root)
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr
    env.update(WORLD_SIZE="2")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--stub-solve"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=root)
    assert r.returncode != 0
