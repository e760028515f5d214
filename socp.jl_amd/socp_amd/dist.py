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
    rec = torch.empty((B, 4), dtype=torch.float64, device=status.device)
    pair = torch.stack([status.to(torch.int32).reshape(-1), iters.to(torch.int32).reshape(-1)], dim=1)
    rec[:, 0] = pair.contiguous().view(torch.float64).reshape(-1)
    if res is None:
        rec[:, 1:] = float("nan")
    else:
        rec[:, 1:] = res.reshape(B, 3).to(torch.float64)
    return rec.view(torch.uint8)


def unpack_outcomes(rec):
    """[..., 32] uint8 records -> dict(status, iters: int32 [...], res: float64 [..., 3])."""
    import torch
    lead = rec.shape[:-1]
    f = rec.contiguous().view(torch.float64).reshape(*lead, 4)
    pair = f[..., 0].contiguous().view(torch.int32).reshape(*lead, 2)
    return {"status": pair[..., 0], "iters": pair[..., 1], "res": f[..., 1:]}


def gather_outcomes(status, iters, res=None, group=None):
    """All-gather every rank's 32-byte outcome records (the path's only exchange
    step); returns dict(status [world, B], iters [world, B],
    res [world, B, 3]).  Equal shard sizes (weak scaling) are required by
    all_gather_into_tensor."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    local = pack_outcomes(status, iters, res).reshape(-1)
    out = torch.empty((world, local.numel()), dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out.view(-1), local, group=group)
    return unpack_outcomes(out.view(world, -1, RECORD_BYTES))


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
