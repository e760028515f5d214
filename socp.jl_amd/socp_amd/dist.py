"""Multi-GPU sharding: independent problems, contiguous global
index ranges per rank, one process per GPU, and a single collective — the
all-gather of each problem's 32-byte outcome record (status, iters, ||rd||,
||rp||, z's: the exit-test quantities of solver.jl:109-122) — over RCCL
(backend "nccl") on MI355X or gloo on the CPU."""
from __future__ import annotations


def shard_range(total: int, rank: int, world: int):
    """Contiguous block [lo, hi) of the global problem index for this rank."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


RECORD_BYTES = 32  # socp_outcome (include/socp.h)


def pack_outcomes(status, iters, res=None):
    """[B, 32] uint8: per problem int32 status, int32 iters, float64 ||rd||, ||rp||,
    z's (socp_outcome layout; NaN residuals when `res` is None)."""
    import torch
    B = status.numel()
    # int32 [B, 8]: slots 0-1 the integers, slots 2-7 the three doubles' bit
    # patterns (int32 views), so no integer bits pass through a floating-point copy
    rec = torch.empty((B, 8), dtype=torch.int32, device=status.device)
    rec[:, 0] = status.reshape(-1).to(torch.int32)
    rec[:, 1] = iters.reshape(-1).to(torch.int32)
    if res is None:
        r = torch.full((B, 3), float("nan"), dtype=torch.float64, device=status.device)
    else:
        r = res.reshape(B, 3).to(torch.float64).contiguous()
    rec[:, 2:] = r.view(torch.int32).reshape(B, 6)
    return rec.view(torch.uint8)


def unpack_outcomes(rec):
    """[..., 32] uint8 records -> dict(status, iters: int32 [...], res: float64 [..., 3])."""
    import torch
    lead = rec.shape[:-1]
    w = rec.contiguous().view(torch.int32).reshape(*lead, 8)
    res = w[..., 2:].contiguous().view(torch.float64).reshape(*lead, 3)
    return {"status": w[..., 0].contiguous(), "iters": w[..., 1].contiguous(), "res": res}


def gather_outcomes(status, iters, res=None, group=None):
    """All-gather every rank's 32-byte outcome records (the path's only exchange
    step); returns dict(status [world, B], iters [world, B],
    res [world, B, 3]).  Equal shard sizes (weak scaling) are required by
    all_gather_into_tensor."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    local = pack_outcomes(status, iters, res).reshape(-1)
    dev = local.device
    if dist.get_backend(group) == "gloo" and dev.type != "cpu":
        local = local.cpu()  # gloo exchanges host buffers (bench.py --dist-backend gloo rehearsal)
    out = torch.empty((world, local.numel()), dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out.view(-1), local, group=group)
    return unpack_outcomes(out.to(dev).view(world, -1, RECORD_BYTES))


COMM_ID_BYTES = 128  # SOCP_COMM_ID_BYTES (include/socp.h)


class StatusComm:
    """The C-ABI RCCL gather (socp_comm_* / socp_allgather_status, include/socp.h):
    what a non-Python host (the Julia shim) uses instead of torch.distributed.
    `uid` is the 128-byte id from `unique_id()` on rank 0, distributed by the host."""

    def __init__(self, ctx, nranks: int, rank: int, uid: bytes):
        import ctypes as C
        from . import _lib
        if len(uid) != COMM_ID_BYTES:
            raise ValueError("uid must be 128 bytes")
        self._L = _lib.load()
        self.ctx, self.nranks, self.rank = ctx, nranks, rank
        self._uid = C.create_string_buffer(bytes(uid), COMM_ID_BYTES)
        h = C.c_void_p()
        _lib.check(self._L.socp_comm_init(ctx.handle, nranks, rank, self._uid, C.byref(h)))
        self.handle = h

    @staticmethod
    def unique_id() -> bytes:
        import ctypes as C
        from . import _lib
        buf = C.create_string_buffer(COMM_ID_BYTES)
        _lib.check(_lib.load().socp_comm_unique_id(buf))
        return buf.raw

    def allgather_status(self, status, iters):
        """int32 [nranks, B, 2] of every rank's (status, iters); device tensors in and out."""
        import torch
        from . import _lib
        B = status.numel()
        self.ctx.bind_torch_stream()  # the conversions below run on torch's stream
        out = torch.empty((self.nranks, B, 2), dtype=torch.int32, device=status.device)
        st = status.to(torch.int32).contiguous()
        it = iters.to(torch.int32).contiguous()
        _lib.check(self._L.socp_allgather_status(self.handle, B, _lib.ptr(st), _lib.ptr(it), _lib.ptr(out)))
        self.ctx.sync()
        return out

    def allgather_outcomes(self, status, iters, res=None):
        """dict(status, iters [nranks, B], res [nranks, B, 3]) of every rank's
        32-byte socp_outcome records (socp_allgather_outcomes); device tensors."""
        import torch
        from . import _lib
        B = status.numel()
        self.ctx.bind_torch_stream()  # the conversions below run on torch's stream
        out = torch.empty((self.nranks, B, RECORD_BYTES), dtype=torch.uint8, device=status.device)
        st = status.to(torch.int32).contiguous()
        it = iters.to(torch.int32).contiguous()
        rs = None if res is None else res.to(torch.float64).contiguous()
        _lib.check(self._L.socp_allgather_outcomes(self.handle, B, _lib.ptr(st), _lib.ptr(it), _lib.ptr(rs),
                                                   _lib.ptr(out)))
        self.ctx.sync()
        return unpack_outcomes(out)

    def close(self):
        if self.handle:
            self._L.socp_comm_destroy(self.handle)
            self.handle = None


def timed_shard_steps(solve_shard, steps: int, warmup: int, sync=None):
    """bench.py's per-rank step loop and accounting (driver contract), for any
    process-group backend (nccl = RCCL on the GPU box, gloo on the CPU).

    solve_shard() -> dict(status, iters, res) solves this rank's shard once; a
    step is that solve plus (world > 1) the all-gather of every problem's
    32-byte outcome record -- the path's only exchange.  W untimed warm-up
    steps, then exactly `steps` steps bracketed by sync() + barrier on both
    sides; the elapsed time is the MAX over ranks and the iteration count the
    SUM over ranks of the problem-iterations each rank executed.

    Returns dict(dt, iters_total, iters_local, out (the last local result),
    gathered (the last gathered records, world > 1), step_ms (per-step wall
    time on this rank))."""
    import time
    import torch
    import torch.distributed as dist
    if steps < 1:
        raise ValueError(f"steps must be >= 1 (got {steps})")
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    sync = sync or (lambda: None)
    st = {"out": None, "gathered": None}

    def step():
        st["out"] = solve_shard()
        if world > 1:
            o = st["out"]
            st["gathered"] = gather_outcomes(o["status"], o["iters"], o.get("res"))

    for _ in range(warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    step_ms = []
    # each step's iteration counts, copied (a device copy for device results:
    # no sync, and a torch reduction inside the loop measured ~14 ms per call
    # on the box) and summed after the timed region
    its = []
    t0 = time.perf_counter()
    for _ in range(steps):
        t1 = time.perf_counter()
        step()
        it_ = st["out"]["iters"]
        its.append(it_.clone() if hasattr(it_, "clone") else it_.copy())
        step_ms.append((time.perf_counter() - t1) * 1e3)
    sync()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    iters_local = 0
    for it_ in its:
        a_ = it_.cpu().numpy() if hasattr(it_, "cpu") else it_
        iters_local += int(a_.astype("int64").sum())
    iters_total = iters_local
    if world > 1:
        dev = st["out"]["iters"].device
        if dist.get_backend() == "gloo":
            dev = torch.device("cpu")
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        it = torch.tensor([iters_local], dtype=torch.int64, device=dev)
        dist.all_reduce(it)
        iters_total = int(it.item())
    return {"dt": dt, "iters_total": iters_total, "iters_local": iters_local, "out": st["out"],
            "gathered": st["gathered"], "step_ms": step_ms}
