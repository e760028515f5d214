"""Multi-GPU sharding: independent problems, contiguous global
index ranges per rank, one process per GPU, and a single collective — the
all-gather of per-problem (status, iters) — over RCCL (backend "nccl") on
MI355X or gloo on the CPU."""
from __future__ import annotations


def shard_range(total: int, rank: int, world: int):
    """Contiguous block [lo, hi) of the global problem index for this rank."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def gather_outcomes(status, iters, group=None):
    """All-gather (status, iters) of every rank's shard; returns int32 [world, B, 2].
    Equal shard sizes (weak scaling) are required by all_gather_into_tensor."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    local = torch.stack([status.to(torch.int32), iters.to(torch.int32)], dim=1).contiguous()
    out = torch.empty((world,) + tuple(local.shape), dtype=torch.int32, device=local.device)
    dist.all_gather_into_tensor(out.view(-1, 2), local, group=group)
    return out


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

    def close(self):
        if self.handle:
            self._L.socp_comm_destroy(self.handle)
            self.handle = None
