"""socp_amd — MI355X-native batched dense SOCP solver (host side).

Two layers over libsocp.so (include/socp.h):

* ``batch_solve`` / ``batch_kkt_solve`` / ``generate``: the batched C-ABI
  entry points, taking numpy arrays (host) or torch CUDA tensors (device).
* A mirror of the reference Julia surface for the dense path
  (BenChung/Socp.jl): ``POC``, ``SOC`` (Socp.jl:9-16), ``Problem``
  (Socp.jl:20-60), ``State`` (Socp.jl:62-75), ``DenseSolver`` (the
  KKTSolver plugin, densesolver.jl:1-90, here running on the GPU),
  ``SolverState`` (solver.jl:1-38), ``solve_socp`` (solver.jl:40-153),
  ``compute_scaling`` / ``setup_iter`` / ``solve_kkt`` with the reference's
  argument meaning and error behaviour (PosDefException from cholesky!,
  DomainError from sqrt of a negative number, AssertionError on shapes).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import (CHOL_H_FAILED, CHOL_S_FAILED, CONE_POC, CONE_SOC, CONVERGED, DOMAIN_ERROR,
                   F_DEVICE_PTRS, F_EXPLICIT_INVERSE, F_FORCE_LARGE, F_WARM_START, MAXIT, Context, SocpError,
                   default_context,
                   default_params)

__all__ = [
    "POC", "SOC", "Problem", "State", "Scaling", "DenseSolver", "HipDenseSolver", "SolverState",
    "solve_socp", "solve_socp_batched", "compute_scaling", "setup_iter", "solve_kkt",
    "PosDefException", "DomainError", "batch_solve", "batch_kkt_solve", "DenseHandle", "Ingest",
    "generate", "pack_csc",
    "Context", "SocpError", "default_context", "cone_arrays",
    "CONVERGED", "MAXIT", "CHOL_H_FAILED", "CHOL_S_FAILED", "DOMAIN_ERROR",
]

STATUS_NAMES = {CONVERGED: "converged", MAXIT: "maxit", CHOL_H_FAILED: "chol(H) failed",
                CHOL_S_FAILED: "chol(S) failed", DOMAIN_ERROR: "domain error"}


class PosDefException(Exception):
    """Raised where the reference's cholesky! throws (densesolver.jl:47,51)."""


class DomainError(Exception):
    """Raised where the reference's sqrt of a negative number throws."""


# ----------------------------------------------------------------- cones
class POC:
    """Nonnegative orthant cone POC(offs, dim) (Socp.jl:9-12)."""

    kind = CONE_POC

    def __init__(self, offs: int, dim: int):
        self.offs, self.dim = int(offs), int(dim)

    def __repr__(self):
        return f"POC({self.offs},{self.dim})"


class SOC:
    """Second-order cone SOC(offs, dim) (Socp.jl:13-16)."""

    kind = CONE_SOC

    def __init__(self, offs: int, dim: int):
        self.offs, self.dim = int(offs), int(dim)

    def __repr__(self):
        return f"SOC({self.offs},{self.dim})"


def _as_cone_list(cones):
    out = []
    for c in cones:
        if isinstance(c, (POC, SOC)):
            out.append((c.kind, c.offs, c.dim))
        else:
            out.append((int(c[0]), int(c[1]), int(c[2])))
    return out


def cone_arrays(cones):
    cl = _as_cone_list(cones)
    kind = np.array([c[0] for c in cl], dtype=np.int32)
    offs = np.array([c[1] for c in cl], dtype=np.int32)
    dim = np.array([c[2] for c in cl], dtype=np.int32)
    return kind, offs, dim


# --------------------------------------------------------------- batched
def _is_torch(a):
    return a is not None and not isinstance(a, np.ndarray) and hasattr(a, "data_ptr")


def _host(a, dtype=np.float64):
    if a is None:
        return None
    return np.ascontiguousarray(a, dtype=dtype)


def _size(a):
    return a.numel() if _is_torch(a) else np.size(a)


def _check_sizes(B, **arrays):
    """Every array must hold exactly its batch-stacked element count (the C ABI
    reads that many elements from each pointer)."""
    if B > _lib.MAX_BATCH:
        raise ValueError(f"batch {B} above 2^31-1")
    for name, (a, want) in arrays.items():
        if a is None:
            continue
        got = _size(a)
        if got != want:
            raise ValueError(f"{name}: {got} elements, expected {want} (batch {B})")


def batch_solve(cones, n, m, k, c, A, b, G, h, sing=None, *, maxit=40, tol=1e-5, step=0.99,
                sigma_exp=3, init_eps=1e-10, warm=None, ctx=None, res=False, out=None, force_large=False,
                explicit_inverse=False):
    """Solve a batch of independent problems (same dims and cone structure).

    Arrays follow include/socp.h: per-problem column-major A (m x n), G (k x n)
    stacked batch-major, vectors stacked batch-major.  numpy inputs run through
    host staging buffers; torch CUDA tensors are used in place (device mode,
    stream-ordered on the context's stream; call ctx.sync() before reading).
    force_large runs the blocked kernel (socp_large.hip) even where the
    register-resident one applies.  explicit_inverse (SOCP_F_EXPLICIT_INVERSE)
    forms Li = H^-1 as densesolver.jl:48 does -- the reference's op order --
    instead of the Cholesky factor + triangular solves of the m <= 16 shapes.
    Returns dict(x, y, z, s, iters, status[, res]).
    """
    L = _lib.load()
    kind, offs, dim = cone_arrays(cones)
    B = _size(c) // n
    if B * n != _size(c):
        raise ValueError(f"c: {_size(c)} elements is not a multiple of n={n}")
    _check_sizes(B, A=(A if m else None, B * m * n), b=(b if m else None, B * m), G=(G, B * k * n),
                 h=(h, B * k), sing=(sing, B))
    if warm is not None:
        wx, wy, wz, ws = warm
        _check_sizes(B, warm_x=(wx, B * n), warm_y=(wy if m else None, B * m), warm_z=(wz, B * k),
                     warm_s=(ws, B * k))
    dims = _lib.Dims(B, n, m, k, len(kind))
    ctx = ctx or default_context()
    dev = _is_torch(G)
    flags = F_DEVICE_PTRS if dev else 0
    if warm is not None:
        flags |= F_WARM_START
    if force_large:
        flags |= F_FORCE_LARGE
    if explicit_inverse:
        flags |= F_EXPLICIT_INVERSE
    P = default_params(maxit=maxit, tol=tol, step=step, sigma_exp=sigma_exp, init_eps=init_eps,
                       flags=flags)
    if dev:
        import torch
        devc = G.device
        ctx.bind_torch_stream()  # ordered after torch's producers of the inputs
        if out is None:
            f64 = dict(dtype=torch.float64, device=devc)
            out = dict(x=torch.empty(B * n, **f64), y=torch.empty(max(B * m, 1), **f64),
                       z=torch.empty(B * k, **f64), s=torch.empty(B * k, **f64),
                       iters=torch.empty(B, dtype=torch.int32, device=devc),
                       status=torch.empty(B, dtype=torch.int32, device=devc))
            if res:
                out["res"] = torch.empty(3 * B, **f64)
        if warm is not None:
            for key, v in zip("xyzs", warm):
                if key == "y" and m == 0:
                    continue
                out[key].copy_(v.reshape(-1))
        arrs = dict(c=c, A=A, b=b, G=G, h=h, sing=sing)
    else:
        out = dict(x=np.zeros(B * n), y=np.zeros(max(B * m, 1)), z=np.zeros(B * k),
                   s=np.zeros(B * k), iters=np.zeros(B, np.int32), status=np.zeros(B, np.int32))
        if res:
            out["res"] = np.zeros(3 * B)
        if warm is not None:
            for key, v in zip("xyzs", warm):
                if key == "y" and m == 0:
                    continue
                out[key][:] = np.asarray(v, dtype=np.float64).reshape(-1)
        arrs = dict(c=_host(c), A=_host(A) if m else None, b=_host(b) if m else None, G=_host(G),
                    h=_host(h), sing=_host(sing, np.uint8) if sing is not None else None)
    p = _lib.ptr
    rc = L.socp_batch_solve_ex(
        ctx.handle, dims, p(kind), p(offs), p(dim), p(arrs["c"]), p(arrs["A"] if m else None),
        p(arrs["b"] if m else None), p(arrs["G"]), p(arrs["h"]), p(arrs["sing"]), P,
        p(out["x"]), p(out["y"] if m else None), p(out["z"]), p(out["s"]), p(out["iters"]),
        p(out["status"]), p(out.get("res")))
    _lib.check(rc)
    if not dev and m == 0:
        out["y"] = out["y"][:0]
    return out


def batch_kkt_solve(cones, n, m, k, A, G, sing, s, z, dx, dy, dz, ds, *, ctx=None, force_large=False,
                    explicit_inverse=False):
    """One KKT solve per problem at iterate (s, z): scaling + setup_iter + solve_kkt
    (densesolver.jl:41-90) on the GPU.  Host (numpy) arrays.  Returns dict(cx,cy,cz,cs,status)."""
    L = _lib.load()
    kind, offs, dim = cone_arrays(cones)
    B = np.size(s) // k
    if B * k != np.size(s):
        raise ValueError(f"s: {np.size(s)} elements is not a multiple of k={k}")
    _check_sizes(B, A=(A if m else None, B * m * n), G=(G, B * k * n), sing=(sing, B), z=(z, B * k),
                 dx=(dx, B * n), dy=(dy if m else None, B * m), dz=(dz, B * k), ds=(ds, B * k))
    dims = _lib.Dims(B, n, m, k, len(kind))
    ctx = ctx or default_context()
    cx, cy, cz, cs = np.zeros(B * n), np.zeros(max(B * m, 1)), np.zeros(B * k), np.zeros(B * k)
    st = np.zeros(B, np.int32)
    p = _lib.ptr
    sg = None if sing is None else _host(sing, np.uint8)
    rc = L.socp_batch_kkt_solve(ctx.handle, dims, p(kind), p(offs), p(dim),
                                p(_host(A) if m else None), p(_host(G)), p(sg), p(_host(s)), p(_host(z)),
                                p(_host(dx)), p(_host(dy) if m else None), p(_host(dz)), p(_host(ds)),
                                p(cx), p(cy if m else None), p(cz), p(cs), p(st),
                                (F_FORCE_LARGE if force_large else 0)
                                | (F_EXPLICIT_INVERSE if explicit_inverse else 0))
    _lib.check(rc)
    return dict(cx=cx, cy=cy[:B * m], cz=cz, cs=cs, status=st)


class DenseHandle:
    """A batch of DenseSolver objects on the device (socp_dense_*): the
    reference's plugin split (densesolver.jl) -- construction keeps A and G
    resident (:19-38), ``setup_iter(s, z)`` computes the NT scaling and the
    factorisation (:41-52) into one record per problem, ``solve_kkt`` solves one
    right-hand side against it (:54-90) as often as called.

    numpy inputs: every call copies its vectors host-to-device (2k doubles per
    problem for setup_iter, n+m+2k for solve_kkt; ``h2d_bytes`` reports the last
    call's count).  torch CUDA inputs (A, G given as tensors): every later
    argument must be a device tensor too; calls are stream-ordered on torch's
    current stream.  Results are bitwise those of ``batch_kkt_solve``."""

    _pfx = "socp_dense"

    def _fn(self, name):
        return getattr(_lib.load(), f"{self._pfx}_{name}")

    def __init__(self, cones, n, m, k, A, G, sing=None, *, ctx=None, force_large=False, explicit_inverse=False):
        self.cones, self.n, self.m, self.k = cones, n, m, k
        self.kind, self.offs, self.dim = cone_arrays(cones)
        B = _size(G) // (k * n)
        if B * k * n != _size(G):
            raise ValueError(f"G: {_size(G)} elements is not a multiple of k*n={k * n}")
        _check_sizes(B, A=(A if m else None, B * m * n), sing=(sing, B))
        self.B = B
        self.ctx = ctx or default_context()
        self.dev = _is_torch(G)
        flags = ((F_DEVICE_PTRS if self.dev else 0) | (F_FORCE_LARGE if force_large else 0)
                 | (F_EXPLICIT_INVERSE if explicit_inverse else 0))
        if self.dev:
            self.ctx.bind_torch_stream()
            arrs = (A if m else None, G, sing)
        else:
            arrs = (_host(A) if m else None, _host(G), None if sing is None else _host(sing, np.uint8))
        h = C.c_void_p()
        dims = _lib.Dims(B, n, m, k, len(self.kind))
        p = _lib.ptr
        _lib.check(self._fn("create")(self.ctx.handle, dims, p(self.kind), p(self.offs), p(self.dim),
                                       p(arrs[0]), p(arrs[1]), p(arrs[2]), flags, C.byref(h)))
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            self._fn("destroy")(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _arg(self, a, dtype=np.float64):
        if self.dev:
            if not _is_torch(a):
                raise TypeError("a device handle takes torch CUDA tensors")
            return a
        return _host(a, dtype)

    def setup_iter(self, s, z, status=None):
        """Scaling + factorisation at (s, z); returns the per-problem status
        (0, CHOL_H_FAILED, CHOL_S_FAILED, DOMAIN_ERROR)."""
        B, k = self.B, self.k
        _check_sizes(B, s=(s, B * k), z=(z, B * k))
        if status is None:
            if self.dev:
                import torch
                status = torch.empty(B, dtype=torch.int32, device=s.device)
            else:
                status = np.zeros(B, np.int32)
        if self.dev:
            self.ctx.bind_torch_stream()
        p = _lib.ptr
        _lib.check(self._fn("setup_iter")(self.handle, p(self._arg(s)), p(self._arg(z)), p(status)))
        return status

    def solve_kkt(self, dx, dy, dz, ds, out=None):
        """One KKT solve per problem against the last setup_iter; returns
        dict(cx, cy, cz, cs, status) (``out`` may supply the arrays)."""
        B, n, m, k = self.B, self.n, self.m, self.k
        _check_sizes(B, dx=(dx, B * n), dy=(dy if m else None, B * m), dz=(dz, B * k), ds=(ds, B * k))
        if out is None:
            if self.dev:
                import torch
                f64 = dict(dtype=torch.float64, device=dz.device)
                out = dict(cx=torch.empty(B * n, **f64), cy=torch.empty(max(B * m, 1), **f64),
                           cz=torch.empty(B * k, **f64), cs=torch.empty(B * k, **f64),
                           status=torch.empty(B, dtype=torch.int32, device=dz.device))
            else:
                out = dict(cx=np.zeros(B * n), cy=np.zeros(max(B * m, 1)), cz=np.zeros(B * k),
                           cs=np.zeros(B * k), status=np.zeros(B, np.int32))
        if self.dev:
            self.ctx.bind_torch_stream()
        p = _lib.ptr
        _lib.check(self._fn("solve_kkt")(
            self.handle, p(self._arg(dx)), p(self._arg(dy) if m else None), p(self._arg(dz)),
            p(self._arg(ds)), p(out["cx"]), p(out["cy"] if m else None), p(out["cz"]), p(out["cs"]),
            p(out["status"])))
        if m == 0 or _size(out["cy"]) != B * m:
            out["cy"] = out["cy"][:B * m]
        return out

    @property
    def h2d_bytes(self) -> int:
        """Host-to-device bytes moved by the last call (socp_dense_h2d_bytes)."""
        v = C.c_int64()
        _lib.check(self._fn("h2d_bytes")(self.handle, C.byref(v)))
        return int(v.value)

    @property
    def record_bytes(self) -> int:
        """Device bytes of one problem's factor record."""
        return int(self._fn("record_bytes")(self.handle))


class SqrHandle(DenseHandle):
    """A batch of SparseSolver objects with SqrScaling on the device
    (socp_sqr_*, the reference's rank-update path: spsolver.jl,
    sqrscalings.jl).  ``setup_iter(s, z)`` computes W^-2 = D + uu' - vv',
    factors G'DG (+A'A), applies one rank-1 update (G'u) and one downdate (G'v)
    per SOC cone and factors S; ``solve_kkt`` solves by triangular solves.
    Same call conventions as DenseHandle; n, m <= 1024, k <= 4096 (one
    wavefront per problem up to n, m = 64, one workgroup above)."""

    _pfx = "socp_sqr"

    def __init__(self, cones, n, m, k, A, G, sing=None, *, ctx=None):
        super().__init__(cones, n, m, k, A, G, sing, ctx=ctx)

    def factor(self, problem: int):
        """The factor L of H after modify_factors! for one problem (n x n lower
        triangular numpy array; L L' = G'W^-2 G (+A'A)) -- the Gfact of spsolver.jl:13."""
        out = np.zeros(self.n * self.n)
        _lib.check(self._fn("factor")(self.handle, int(problem), _lib.ptr(out)))
        return out.reshape(self.n, self.n, order="F")

    def solve_socp(self, c, b, h, *, maxit=40, tol=1e-5, step=0.99, sigma_exp=3, init_eps=1e-10, res=True):
        """solve_socp(prob, SolverState(prob, SparseSolver(prob))) (solver.jl:40-153)
        for every problem of the batch, on this plugin (socp_sqr_solve_socp):
        the reference's own tested path, batched.  Returns dict(x, y, z, s,
        iters, status[, res]) like ``batch_solve``; numpy or torch as the handle."""
        B, n, m, k = self.B, self.n, self.m, self.k
        _check_sizes(B, c=(c, B * n), b=(b if m else None, B * m), h=(h, B * k))
        if self.dev:
            import torch
            dv = c.device
            f64 = dict(dtype=torch.float64, device=dv)
            out = dict(x=torch.empty(B * n, **f64), y=torch.empty(max(B * m, 1), **f64),
                       z=torch.empty(B * k, **f64), s=torch.empty(B * k, **f64),
                       iters=torch.empty(B, dtype=torch.int32, device=dv),
                       status=torch.empty(B, dtype=torch.int32, device=dv))
            if res:
                out["res"] = torch.empty(3 * B, **f64)
            self.ctx.bind_torch_stream()
        else:
            out = dict(x=np.zeros(B * n), y=np.zeros(max(B * m, 1)), z=np.zeros(B * k), s=np.zeros(B * k),
                       iters=np.zeros(B, np.int32), status=np.zeros(B, np.int32))
            if res:
                out["res"] = np.zeros(3 * B)
        P = _lib.default_params(maxit=maxit, tol=tol, step=step, sigma_exp=sigma_exp, init_eps=init_eps)
        p = _lib.ptr
        _lib.check(self._fn("solve_socp")(self.handle, p(self._arg(c)), p(self._arg(b)) if m else None,
                                           p(self._arg(h)), C.byref(P), p(out["x"]), p(out["y"]) if m else None,
                                           p(out["z"]), p(out["s"]), p(out["iters"]), p(out["status"]),
                                           p(out.get("res"))))
        out["y"] = out["y"][:B * m]
        return out

    def scaling(self):
        """dict(l, wbs, mu) of the last setup_iter for every problem (host arrays
        B x k, B x k, B x ncones): the SqrScaling fields the driver loop reads."""
        B, k, nc = self.B, self.k, len(self.kind)
        l, wbs, mu = np.zeros(B * k), np.zeros(B * k), np.zeros(B * nc)
        _lib.check(self._fn("scaling")(self.handle, _lib.ptr(l), _lib.ptr(wbs), _lib.ptr(mu)))
        return dict(l=l.reshape(B, k), wbs=wbs.reshape(B, k), mu=mu.reshape(B, nc))


def sqr_supported(n, m, k, ncones) -> bool:
    """Whether the rank-update plugin takes these dims (socp_sqr_supported)."""
    return bool(_lib.load().socp_sqr_supported(_lib.Dims(1, n, m, k, ncones)))


def _csc_arrays(mats, rows, cols, index_base):
    """(nz_offs, colptr, rowval, nzval) host arrays of a list of scipy.sparse
    matrices in canonical CSC form (sorted, duplicates summed)."""
    csc = []
    for M in mats:
        M = M.tocsc(copy=True)
        M.sum_duplicates()
        if M.shape != (rows, cols):
            raise ValueError(f"matrix shape {M.shape}, expected {(rows, cols)}")
        csc.append(M)
    nz = np.cumsum(np.array([0] + [M.nnz for M in csc], dtype=np.int64))
    colptr = (np.concatenate([M.indptr.astype(np.int64) + index_base for M in csc]) if csc
              else np.zeros(1, np.int64))
    rowval = (np.concatenate([M.indices.astype(np.int64) + index_base for M in csc]) if nz[-1]
              else np.zeros(1, np.int64))
    nzval = np.concatenate([M.data.astype(np.float64) for M in csc]) if nz[-1] else np.zeros(1)
    return nz, colptr, rowval, nzval


class Ingest:
    """Pipelined host ingest (socp_ingest_*): host batches through two slots of
    pinned staging, batch i+1's host-to-device copy (and CSC packing) overlapping
    batch i's solve.  ``submit`` / ``submit_csc`` return a ticket, ``wait``
    returns the batch_solve dict; at most two tickets are outstanding.
    ``next_inputs()`` gives numpy views of the next slot's pinned input arrays
    (a producer filling them in place saves the host copy)."""

    def __init__(self, cones, n, m, k, max_batch, *, ctx=None, force_large=False):
        L = _lib.load()
        self.cones, self.n, self.m, self.k, self.max_batch = cones, n, m, k, int(max_batch)
        self.kind, self.offs, self.dim = cone_arrays(cones)
        self.ctx = ctx or default_context()
        h = C.c_void_p()
        dims = _lib.Dims(self.max_batch, n, m, k, len(self.kind))
        p = _lib.ptr
        _lib.check(L.socp_ingest_create(self.ctx.handle, dims, p(self.kind), p(self.offs), p(self.dim),
                                        F_FORCE_LARGE if force_large else 0, C.byref(h)))
        self.handle = h
        self._batch = {}

    def close(self):
        if getattr(self, "handle", None):
            _lib.load().socp_ingest_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def next_inputs(self):
        ptrs = [C.c_void_p() for _ in range(6)]
        _lib.check(_lib.load().socp_ingest_next_inputs(self.handle, *[C.byref(q) for q in ptrs]))
        B, n, m, k = self.max_batch, self.n, self.m, self.k
        out = {}
        for key, q, cnt, ct in zip(("c", "A", "b", "G", "h", "sing"), ptrs,
                                   (B * n, B * m * n, B * m, B * k * n, B * k, B),
                                   (C.c_double,) * 5 + (C.c_uint8,)):
            out[key] = np.ctypeslib.as_array(C.cast(q, C.POINTER(ct)), shape=(max(cnt, 1),))[:cnt]
        return out

    def _params(self, maxit, tol, step, sigma_exp, init_eps):
        return default_params(maxit=maxit, tol=tol, step=step, sigma_exp=sigma_exp, init_eps=init_eps)

    def submit(self, c, A, b, G, h, sing=None, *, maxit=40, tol=1e-5, step=0.99, sigma_exp=3, init_eps=1e-10):
        n, m, k = self.n, self.m, self.k
        B = np.size(c) // n
        _check_sizes(B, c=(c, B * n), A=(A if m else None, B * m * n), b=(b if m else None, B * m),
                     G=(G, B * k * n), h=(h, B * k), sing=(sing, B))
        t = C.c_int64()
        P = self._params(maxit, tol, step, sigma_exp, init_eps)
        p = _lib.ptr
        arr = [_host(c), _host(A) if m else None, _host(b) if m else None, _host(G), _host(h),
               None if sing is None else _host(sing, np.uint8)]
        _lib.check(_lib.load().socp_ingest_submit(self.handle, B, *[p(a) for a in arr], P, C.byref(t)))
        self._batch[t.value] = B
        return t.value

    def submit_csc(self, c, b, h, sing, A_mats, G_mats, *, index_base=1, maxit=40, tol=1e-5, step=0.99,
                   sigma_exp=3, init_eps=1e-10):
        """A_mats, G_mats: lists of scipy.sparse matrices (m x n, k x n), or
        tuples (nz_offs, colptr, rowval, nzval) of host arrays."""
        n, m, k = self.n, self.m, self.k
        B = np.size(c) // n
        _check_sizes(B, c=(c, B * n), b=(b if m else None, B * m), h=(h, B * k), sing=(sing, B))
        Acsc = (A_mats if isinstance(A_mats, tuple) else _csc_arrays(A_mats, m, n, index_base)) if m else None
        Gcsc = G_mats if isinstance(G_mats, tuple) else _csc_arrays(G_mats, k, n, index_base)
        Acsc = [np.ascontiguousarray(a) for a in Acsc] if Acsc is not None else [None] * 4
        Gcsc = [np.ascontiguousarray(a) for a in Gcsc]
        t = C.c_int64()
        P = self._params(maxit, tol, step, sigma_exp, init_eps)
        p = _lib.ptr
        _lib.check(_lib.load().socp_ingest_submit_csc(
            self.handle, B, p(_host(c)), p(_host(b) if m else None), p(_host(h)),
            p(None if sing is None else _host(sing, np.uint8)), *[p(a) for a in Acsc], *[p(a) for a in Gcsc],
            index_base, P, C.byref(t)))
        self._batch[t.value] = B
        return t.value

    def wait(self, ticket, res=False):
        B = self._batch.pop(ticket, None)
        if B is None:
            raise ValueError(f"unknown ticket {ticket}")
        n, m, k = self.n, self.m, self.k
        out = dict(x=np.zeros(B * n), y=np.zeros(max(B * m, 1)), z=np.zeros(B * k), s=np.zeros(B * k),
                   iters=np.zeros(B, np.int32), status=np.zeros(B, np.int32))
        if res:
            out["res"] = np.zeros(3 * B)
        p = _lib.ptr
        _lib.check(_lib.load().socp_ingest_wait(self.handle, ticket, p(out["x"]), p(out["y"] if m else None),
                                                p(out["z"]), p(out["s"]), p(out["iters"]), p(out["status"]),
                                                p(out.get("res"))))
        out["y"] = out["y"][:B * m]
        return out


def generate(cones, B, n, m, k, seed, first_problem=0, *, ctx=None, device=None):
    """Device-side generation of B feasible synthetic problems;
    returns torch CUDA tensors (c, A, b, G, h) in the include/socp.h layout."""
    import torch
    ctx = ctx or default_context()
    dev = device or torch.device("cuda", ctx.device)
    f64 = dict(dtype=torch.float64, device=dev)
    c, A, b = torch.empty(B * n, **f64), torch.empty(max(B * m * n, 1), **f64), torch.empty(max(B * m, 1), **f64)
    G, h = torch.empty(B * k * n, **f64), torch.empty(B * k, **f64)
    kind, offs, dim = cone_arrays(cones)
    dims = _lib.Dims(B, n, m, k, len(kind))
    p = _lib.ptr
    ctx.bind_torch_stream()
    _lib.check(_lib.load().socp_generate(ctx.handle, dims, p(kind), p(offs), p(dim), seed,
                                         first_problem, p(c), p(A), p(b), p(G), p(h)))
    return c, A[:B * m * n], b[:B * m], G, h


def pack_csc(mats, rows=None, cols=None, *, index_base=1, ctx=None, device=None):
    """Ingest: pack sparse matrices in SparseMatrixCSC form --
    the storage of Problem.A / Problem.G (Socp.jl:25,29) -- into the dense
    column-major batch layout on the device (socp_pack_csc).  `mats` is a list
    of scipy.sparse matrices (CSC after conversion), or a tuple of device int64
    tensors (nz_offs, colptr, rowval) plus a float64 nzval tensor with rows, cols
    given.  Returns a flat torch float64 tensor of B*rows*cols."""
    import torch
    ctx = ctx or default_context()
    dev = device or torch.device("cuda", ctx.device)
    if isinstance(mats, tuple):
        nz_offs, colptr, rowval, nzval = mats
        B = nz_offs.numel() - 1
    else:
        # canonical CSC (sorted row indices, duplicates summed in order, as
        # Julia's sparse() stores them); the device kernel also sums unsorted
        # or repeated entries, but only this form is bitwise reproducible
        csc = []
        for m in mats:
            m = m.tocsc(copy=True)
            m.sum_duplicates()
            csc.append(m)
        B = len(csc)
        rows, cols = csc[0].shape if B else (rows or 0, cols or 0)
        for m in csc:
            assert m.shape == (rows, cols)
        nnz = np.array([0] + [m.nnz for m in csc], dtype=np.int64)
        nz = np.cumsum(nnz)
        i64 = dict(dtype=torch.int64, device=dev)
        nz_offs = torch.tensor(nz, **i64)
        colptr = torch.tensor(np.concatenate([m.indptr.astype(np.int64) + index_base for m in csc])
                              if B else np.zeros(0, np.int64), **i64)
        rowval = torch.tensor(np.concatenate([m.indices.astype(np.int64) + index_base for m in csc])
                              if B and nz[-1] else np.zeros(1, np.int64), **i64)
        nzval = torch.tensor(np.concatenate([m.data.astype(np.float64) for m in csc])
                             if B and nz[-1] else np.zeros(1), dtype=torch.float64, device=dev)
    out = torch.empty(max(B * rows * cols, 1), dtype=torch.float64, device=dev)
    p = _lib.ptr
    ctx.bind_torch_stream()
    _lib.check(_lib.load().socp_pack_csc(ctx.handle, B, rows, cols, p(nz_offs), p(colptr), p(rowval),
                                         p(nzval), index_base, p(out)))
    return out[:B * rows * cols]


# ------------------------------------------------- reference-shaped mirror
def _colmajor(M, rows, cols):
    M = np.asarray(M, dtype=np.float64).reshape(rows, cols) if rows * cols else np.zeros((rows, cols))
    return np.ascontiguousarray(M.ravel(order="F"))


class Problem:
    """Problem(c, A, b, G, h, cones) (Socp.jl:40-59).  `sing` is true when
    cholesky(G'G) throws, exactly the reference's rule (Socp.jl:49-56)."""

    def __init__(self, c, A, b, G, h, cones):
        c = np.asarray(c, dtype=np.float64).reshape(-1)
        n = len(c)
        A = np.asarray(A, dtype=np.float64)
        A = A.reshape(-1, n) if A.size else np.zeros((0, n))
        b = np.asarray(b, dtype=np.float64).reshape(-1)
        G = np.asarray(G, dtype=np.float64)
        h = np.asarray(h, dtype=np.float64).reshape(-1)
        m = A.shape[0]
        assert len(b) == m
        assert A.shape[1] == n
        assert G.shape[1] == n
        k = G.shape[0]
        assert len(h) == k
        self.c, self.A, self.b, self.G, self.h = c, A, b, G, h
        self.cones = tuple(cones)
        self.n, self.m, self.k = n, m, k
        try:
            np.linalg.cholesky(G.T @ G)
            self.sing = False
        except np.linalg.LinAlgError:
            self.sing = True


class State:
    """State(prob, x, y, z, s) (Socp.jl:62-75)."""

    def __init__(self, prob: Problem, x, y, z, s):
        self.x = np.array(x, dtype=np.float64).reshape(-1)
        self.y = np.array(y, dtype=np.float64).reshape(-1)
        self.z = np.array(z, dtype=np.float64).reshape(-1)
        self.s = np.array(s, dtype=np.float64).reshape(-1)
        assert len(self.x) == prob.n
        assert len(self.y) == prob.m
        assert len(self.z) == prob.k
        assert len(self.s) == prob.k


class Scaling:
    """NT scaling handle (scalings.jl:1-20), the plugin's AbstractScaling.  The
    scaling W, W^-1, lambda itself lives on the device, in the DenseSolver's
    factor record; this object records the (s, z) compute_scaling was given."""

    def __init__(self, prob: Problem):
        self.s = np.zeros(prob.k)
        self.z = np.zeros(prob.k)


def compute_scaling(cones, scaling: Scaling, s, z):
    """compute_scaling(cones, scaling, s, z) (scalings.jl:101-110).  The
    arithmetic runs on the GPU in the next setup_iter (it feeds only that)."""
    scaling.s = np.array(s, dtype=np.float64)
    scaling.z = np.array(z, dtype=np.float64)
    return scaling


class DenseSolver:
    """KKTSolver{Scaling} plugin for the dense path (densesolver.jl:1-90) on
    MI355X: DenseSolver(pr) (:19-38) keeps A and G on the device (a one-problem
    DenseHandle); setup_iter factors into the handle's record, solve_kkt solves
    against it, so only n+m+2k doubles move per solve."""

    scaling_type = Scaling

    def __init__(self, prob: Problem, ctx: Context | None = None):
        self.prob = prob
        self.ctx = ctx
        self.handle = DenseHandle(prob.cones, prob.n, prob.m, prob.k, _colmajor(prob.A, prob.m, prob.n),
                                  _colmajor(prob.G, prob.k, prob.n), np.array([prob.sing], np.uint8),
                                  ctx=ctx)


HipDenseSolver = DenseSolver


class SqrScaling(Scaling):
    """SqrScaling (sqrscalings.jl:8-48), the scaling type of SparseSolver: the
    factored W^-2 = D + uu' - vv' is computed on the device by setup_iter; this
    object records (s, z) and, after setup_iter, holds the fields the driver
    loop reads (l, wbs, mu), read back from the device."""

    def __init__(self, prob: Problem):
        super().__init__(prob)
        self.l = np.zeros(prob.k)
        self.wbs = np.zeros(prob.k)
        self.mu = np.zeros(len(prob.cones))


class SparseSolver(DenseSolver):
    """KKTSolver{SqrScaling} plugin (spsolver.jl:1-130) on MI355X: the
    rank-update path -- G'DG factored, one rank-1 update and one downdate per
    SOC cone, triangular solves (a one-problem SqrHandle).  The reference runs
    it through CHOLMOD; here the factor is dense and LDS-resident.  The plugin
    methods are setup_iter / solve_kkt; solve_socp with this plugin runs the
    reference's IPM loop on the device with these same kernels
    (SqrHandle.solve_socp, socp_sqr_solve_socp)."""

    scaling_type = SqrScaling

    def __init__(self, prob: Problem, ctx: Context | None = None):
        self.prob = prob
        self.ctx = ctx
        self.handle = SqrHandle(prob.cones, prob.n, prob.m, prob.k, _colmajor(prob.A, prob.m, prob.n),
                                _colmajor(prob.G, prob.k, prob.n), np.array([prob.sing], np.uint8), ctx=ctx)


HipSqrSolver = SparseSolver


def setup_iter(solver: DenseSolver, prob: Problem, state: State, scaling: Scaling):
    """setup_iter(::DenseSolver, ...) (densesolver.jl:41-52): scaling, H, H^-1,
    A H^-1 A' and its factorisation, kept on the device.  Raises
    PosDefException where cholesky! throws, DomainError where the scaling's
    sqrt does."""
    st = solver.handle.setup_iter(scaling.s, scaling.z)
    _raise_status(int(st[0]))
    if isinstance(scaling, SqrScaling) and isinstance(solver.handle, SqrHandle):
        sc = solver.handle.scaling()
        scaling.l, scaling.wbs, scaling.mu = sc["l"][0], sc["wbs"][0], sc["mu"][0]


def _raise_status(st):
    if st in (CHOL_H_FAILED, CHOL_S_FAILED):
        raise PosDefException(STATUS_NAMES[st])
    if st == DOMAIN_ERROR:
        raise DomainError(STATUS_NAMES[st])


def solve_kkt(solver: DenseSolver, prob: Problem, state: State, scaling: Scaling, dx, dy, dz, ds,
              cx, cy, cz, cs):
    """solve_kkt(::DenseSolver, ...) (densesolver.jl:54-90) against the last
    setup_iter: writes (cx,cy,cz,cs) in place, leaves (dx,dy,dz,ds) untouched."""
    out = solver.handle.solve_kkt(dx, dy, dz, ds)
    _raise_status(int(out["status"][0]))
    cx[:] = out["cx"]
    cy[:] = out["cy"]
    cz[:] = out["cz"]
    cs[:] = out["cs"]


class SolverState:
    """SolverState(prob, solver) (solver.jl:22-37): the scaling type comes from
    the plugin (KKTSolver{S} -> S(pr)).  `maxit`, `tol` default to the reference
    constants; after a solve `iters` and `status` hold the outcome."""

    def __init__(self, prob: Problem, solver: DenseSolver, maxit=40, tol=1e-5):
        self.scaling = solver.scaling_type(prob)
        self.solver = solver
        self.maxit, self.tol = maxit, tol
        self.iters, self.status = 0, None


def solve_socp(prob: Problem, ss: SolverState) -> State:
    """solve_socp(prob, ss) (solver.jl:40-153) on the GPU.  Like the reference it
    returns the final State, and raises where the reference throws."""
    if isinstance(ss.solver, SparseSolver):  # the rank-update plugin's own IPM (spsolver.jl)
        out = ss.solver.handle.solve_socp(prob.c, prob.b if prob.m else None, prob.h, maxit=ss.maxit, tol=ss.tol)
    else:
        out = batch_solve(prob.cones, prob.n, prob.m, prob.k, prob.c, _colmajor(prob.A, prob.m, prob.n),
                          prob.b, _colmajor(prob.G, prob.k, prob.n), prob.h,
                          np.array([prob.sing], np.uint8), maxit=ss.maxit, tol=ss.tol,
                          ctx=ss.solver.ctx)
    ss.iters, ss.status = int(out["iters"][0]), int(out["status"][0])
    _raise_status(ss.status)
    return State(prob, out["x"], out["y"], out["z"], out["s"])


def solve_socp_batched(problems, maxit=40, tol=1e-5, ctx=None, solver="dense"):
    """Batched solve of Problems sharing dims and cones; returns (states, iters, status)
    without raising: failures are reported per problem.  solver="dense": the
    DenseSolver path (the fused register / blocked kernels); "sqr": the
    SparseSolver rank-update path (SqrHandle.solve_socp)."""
    p0 = problems[0]
    n, m, k = p0.n, p0.m, p0.k
    for p in problems:
        assert (p.n, p.m, p.k) == (n, m, k)
    c = np.concatenate([p.c for p in problems])
    A = np.concatenate([_colmajor(p.A, m, n) for p in problems]) if m else None
    b = np.concatenate([p.b for p in problems]) if m else None
    G = np.concatenate([_colmajor(p.G, k, n) for p in problems])
    h = np.concatenate([p.h for p in problems])
    sing = np.array([p.sing for p in problems], np.uint8)
    if solver == "sqr":
        out = SqrHandle(p0.cones, n, m, k, A, G, sing, ctx=ctx).solve_socp(c, b, h, maxit=maxit, tol=tol)
    else:
        out = batch_solve(p0.cones, n, m, k, c, A, b, G, h, sing, maxit=maxit, tol=tol, ctx=ctx)
    states = [State(p, out["x"][i * n:(i + 1) * n], out["y"][i * m:(i + 1) * m],
                    out["z"][i * k:(i + 1) * k], out["s"][i * k:(i + 1) * k])
              for i, p in enumerate(problems)]
    return states, out["iters"], out["status"]
