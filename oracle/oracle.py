"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU oracle (socp_oracle.c).

The oracle restates the reference dense path of BenChung/Socp.jl
(src/solver.jl, scalings.jl, vectors.jl, mats.jl, densesolver.jl) in C, in
the reference's op order.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module; the product (socp_amd / libsocp.so)
never does.

Parity pinning: tests/test_oracle.py checks this oracle against every
known-answer vector of the reference's test/runtests.jl, transcribed in
tests/golden/reference_kats.json.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SOCP_ORACLE_LIB: another build of the same source (e.g. build/liboracle_asan.so, `make asan-test`)
_LIB_PATH = os.environ.get("SOCP_ORACLE_LIB") or os.path.join(_HERE, "build", "liboracle.so")

POC, SOC = 0, 1

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_u8 = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


class Params(C.Structure):
    """Mirror of socp_params (include/socp.h); defaults = reference constants."""

    _fields_ = [
        ("maxit", C.c_int32),
        ("sigma_exp", C.c_int32),
        ("tol", C.c_double),
        ("step", C.c_double),
        ("init_eps", C.c_double),
        ("flags", C.c_int32),
        ("reserved", C.c_int32),
    ]

    def __init__(self, maxit=40, tol=1e-5, step=0.99, sigma_exp=3, init_eps=1e-10, flags=0):
        super().__init__(maxit, sigma_exp, tol, step, init_eps, flags, 0)


F_WARM_START = 2
F_STRUCTURED = 16  # oracle-only: the build's structured algorithm (CPU baseline line)
F_CHOLSOLVE = 64  # oracle-only, with F_STRUCTURED: Li v by triangular solves, S = Z'Z (the register kernel at m <= 16)
F_INV_YTY = 128  # oracle-only, with F_STRUCTURED: Li = Y'Y, Y = L^-1 (the kernels' explicit inverse; potrs(I) without it)
F_SQR = 32  # oracle-only: SqrScaling + SparseSolver (spsolver.jl, the rank-update path)


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        cones = [C.c_int, _ip, _ip, _ip]
        L.or_make_e.argtypes = cones + [_dp]
        L.or_vprod.argtypes = cones + [_dp, _dp, _dp]
        L.or_iprod.argtypes = cones + [_dp, _dp, _dp]
        L.or_cgt.argtypes = cones + [_dp, _dp]
        L.or_cgt.restype = C.c_int
        L.or_deg.argtypes = cones
        L.or_deg.restype = C.c_int
        L.or_max_step.argtypes = cones + [_dp]
        L.or_max_step.restype = C.c_double
        L.or_compute_step.argtypes = cones + [_dp, _dp, _dp, C.POINTER(C.c_int)]
        L.or_compute_step.restype = C.c_double
        L.or_compute_scaling.argtypes = cones + [C.c_int, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _dp]
        L.or_compute_scaling.restype = C.c_int
        L.or_scale.argtypes = cones + [_dp, _dp, _dp, _dp, C.c_int]
        L.or_kkt_single.argtypes = (cones + [C.c_int] * 3 + [_dp, _dp, C.c_int] + [_dp] * 6 + [_dp] * 4
                                    + [C.c_void_p, C.c_void_p, C.c_int])
        L.or_kkt_single.restype = C.c_int
        L.or_sqr_kkt_single.argtypes = cones + [C.c_int] * 3 + [_dp, _dp, C.c_int] + [_dp] * 6 + [_dp] * 4 + [C.c_void_p] * 4
        L.or_sqr_kkt_single.restype = C.c_int
        L.or_batch_solve.argtypes = [C.c_int64, C.c_int, C.c_int, C.c_int] + cones + [_dp] * 5 + [C.c_void_p, C.POINTER(Params)] + [_dp] * 4 + [_ip, _ip, C.c_void_p, C.c_int]
        L.or_batch_solve.restype = C.c_int
        L.or_solve_trace.argtypes = [C.c_int] * 3 + cones + [_dp] * 5 + [C.c_int, C.POINTER(Params)] + [_dp] * 4 + [C.POINTER(C.c_int32), C.POINTER(C.c_int32), _dp, _dp, C.c_int]
        L.or_solve_trace.restype = C.c_int
        L.or_init_point.argtypes = [C.c_int] * 3 + cones + [_dp] * 5 + [C.POINTER(Params)] + [_dp] * 4
        L.or_init_point.restype = C.c_int
        L.or_sing.argtypes = [C.c_int, C.c_int, _dp]
        L.or_sing.restype = C.c_int
        L.or_generate.argtypes = [C.c_int64, C.c_int, C.c_int, C.c_int] + cones + [C.c_uint64, C.c_int64] + [_dp] * 5
        _lib = L
    return _lib


def cone_arrays(cones):
    """cones: list of (kind, offs, dim) -> (nc, kind, offs, dim) int32 arrays."""
    kind = np.array([c[0] for c in cones], dtype=np.int32)
    offs = np.array([c[1] for c in cones], dtype=np.int32)
    dim = np.array([c[2] for c in cones], dtype=np.int32)
    return len(cones), kind, offs, dim


def _f(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def make_e(cones, k):
    r = np.zeros(k)
    lib().or_make_e(*cone_arrays(cones), r)
    return r


def vprod(cones, u, v):
    t = np.zeros(len(u))
    lib().or_vprod(*cone_arrays(cones), t, _f(u), _f(v))
    return t


def iprod(cones, lam, v):
    t = np.zeros(len(v))
    lib().or_iprod(*cone_arrays(cones), t, _f(lam), _f(v))
    return t


def cgt(cones, x, dx):
    return bool(lib().or_cgt(*cone_arrays(cones), _f(x), _f(dx)))


def deg(cones):
    return lib().or_deg(*cone_arrays(cones))


def max_step(cones, x):
    return lib().or_max_step(*cone_arrays(cones), _f(x))


def compute_step(cones, l, ds, dz):
    dom = C.c_int(0)
    v = lib().or_compute_step(*cone_arrays(cones), _f(l), _f(ds), _f(dz), C.byref(dom))
    return v, dom.value


def compute_scaling(cones, s, z):
    """Returns dict(W, iW, iWiW, l, mu, wbs, status) as scalings.jl:101-110."""
    k = len(s)
    W, iW, iWiW = (np.zeros(k * k) for _ in range(3))
    l, wbs = np.zeros(k), np.zeros(k)
    mu = np.zeros(max(len(cones), 1))
    st = lib().or_compute_scaling(*cone_arrays(cones), k, _f(s), _f(z), W, iW, iWiW, l, mu, wbs)
    return dict(W=W.reshape(k, k, order="F"), iW=iW.reshape(k, k, order="F"),
                iWiW=iWiW.reshape(k, k, order="F"), l=l, mu=mu, wbs=wbs, status=st)


def scale(cones, wbs, mu, x, inverse=False):
    out = np.zeros(len(x))
    lib().or_scale(*cone_arrays(cones), _f(wbs), _f(mu), _f(x), out, int(inverse))
    return out


def kkt_single(cones, A, G, sing, s, z, dx, dy, dz, ds, want_H=False, structured=False, chol=False):
    """compute_scaling + setup_iter + solve_kkt (densesolver.jl:41-90) at iterate (s,z).
    structured: the kernels' order (X = W^-1 G per cone, H = X'X; F_STRUCTURED)
    instead of the reference's (dense iW*iW', G'*iWiW*G); no H output then.
    chol (with structured): no explicit Li -- Z = L^-1 A', S = Z'Z and the
    triangular solves the register kernel runs for m <= 16 (F_CHOLSOLVE)."""
    A = np.asarray(A, dtype=np.float64).reshape(-1, G.shape[1]) if np.size(A) else np.zeros((0, G.shape[1]))
    m, n = A.shape
    k = G.shape[0]
    cx, cy, cz, cs = np.zeros(n), np.zeros(m), np.zeros(k), np.zeros(k)
    H = np.zeros(n * n) if want_H else None
    Li = np.zeros(n * n) if want_H else None
    st = lib().or_kkt_single(*cone_arrays(cones), n, m, k, _f(A.ravel(order="F")) if m else np.zeros(1),
                             _f(G.ravel(order="F")), int(sing), _f(s), _f(z), _f(dx),
                             _f(dy) if m else np.zeros(1), _f(dz), _f(ds), cx, cy if m else np.zeros(1), cz, cs,
                             H.ctypes.data if want_H else None, Li.ctypes.data if want_H else None,
                             int(bool(structured)) | (2 if (structured and chol) else 0))
    out = dict(cx=cx, cy=cy, cz=cz, cs=cs, status=st)
    if want_H:
        out["H"] = H.reshape(n, n, order="F")
        out["Li"] = Li.reshape(n, n, order="F")
    return out


def sqr_kkt_single(cones, A, G, sing, s, z, dx, dy, dz, ds):
    """SqrScaling + setup_iter + solve_kkt of the rank-update path (sqrscalings.jl:66-194,
    spsolver.jl:60-130) at iterate (s,z).  Returns dict(cx,cy,cz,cs,status,L,l,wbs,mu);
    L is the lower factor of H after modify_factors! (L L' = G'W^-2 G (+A'A))."""
    A = np.asarray(A, dtype=np.float64).reshape(-1, G.shape[1]) if np.size(A) else np.zeros((0, G.shape[1]))
    m, n = A.shape
    k = G.shape[0]
    cx, cy, cz, cs = np.zeros(n), np.zeros(m), np.zeros(k), np.zeros(k)
    Lf, l, wbs, mu = np.zeros(n * n), np.zeros(k), np.zeros(k), np.zeros(len(cones))
    st = lib().or_sqr_kkt_single(*cone_arrays(cones), n, m, k, _f(A.ravel(order="F")) if m else np.zeros(1),
                                 _f(G.ravel(order="F")), int(sing), _f(s), _f(z), _f(dx),
                                 _f(dy) if m else np.zeros(1), _f(dz), _f(ds), cx, cy if m else np.zeros(1), cz, cs,
                                 Lf.ctypes.data, l.ctypes.data, wbs.ctypes.data, mu.ctypes.data)
    return dict(cx=cx, cy=cy, cz=cz, cs=cs, status=st, L=Lf.reshape(n, n, order="F"), l=l, wbs=wbs, mu=mu)


def sing_flag(G):
    k, n = G.shape
    return bool(lib().or_sing(n, k, _f(np.asarray(G).ravel(order="F"))))


def _prob_arrays(c, A, b, G, h):
    n = len(c)
    A = np.asarray(A, dtype=np.float64).reshape(-1, n)
    m = A.shape[0]
    G = np.asarray(G, dtype=np.float64)
    k = G.shape[0]
    Af = _f(A.ravel(order="F")) if m else np.zeros(1)
    bf = _f(b) if m else np.zeros(1)
    return n, m, k, _f(c), Af, bf, _f(G.ravel(order="F")), _f(h)


def solve_trace(cones, c, A, b, G, h, sing=None, params=None, max_trace=41, warm=None):
    """solve_socp (solver.jl:40-153) for one problem with a per-iteration trace.
    Returns dict(x,y,z,s,iters,status,res,trace[t] = (x,y,z,s) at the start of iteration t)."""
    n, m, k, cf, Af, bf, Gf, hf = _prob_arrays(c, A, b, G, h)
    if sing is None:
        sing = sing_flag(np.asarray(G, dtype=np.float64))
    P = params or Params()
    x, y, z, s = np.zeros(n), np.zeros(max(m, 1)), np.zeros(k), np.zeros(k)
    if warm is not None:
        x[:] = warm[0]
        y[:m] = warm[1]
        z[:] = warm[2]
        s[:] = warm[3]
        P = Params(P.maxit, P.tol, P.step, P.sigma_exp, P.init_eps, P.flags | F_WARM_START)
    it, st = C.c_int32(0), C.c_int32(0)
    res = np.zeros(3)
    stride = n + m + 2 * k
    tr = np.zeros(max_trace * stride)
    lib().or_solve_trace(n, m, k, *cone_arrays(cones), cf, Af, bf, Gf, hf, int(sing), C.byref(P),
                         x, y, z, s, C.byref(it), C.byref(st), res, tr, max_trace)
    ntr = min(max_trace, it.value + 1)
    trace = []
    for t in range(ntr):
        v = tr[t * stride:(t + 1) * stride]
        trace.append((v[:n].copy(), v[n:n + m].copy(), v[n + m:n + m + k].copy(), v[n + m + k:].copy()))
    return dict(x=x, y=y[:m], z=z, s=s, iters=it.value, status=st.value, res=res, trace=trace)


def init_point(cones, c, A, b, G, h, params=None):
    n, m, k, cf, Af, bf, Gf, hf = _prob_arrays(c, A, b, G, h)
    x, y, z, s = np.zeros(n), np.zeros(max(m, 1)), np.zeros(k), np.zeros(k)
    st = lib().or_init_point(n, m, k, *cone_arrays(cones), cf, Af, bf, Gf, hf, C.byref(params or Params()), x, y, z, s)
    return dict(x=x, y=y[:m], z=z, s=s, status=st)


def batch_solve(cones, n, m, k, c, A, b, G, h, sing=None, params=None, nthreads=0, warm=None):
    """Batched oracle solve; arrays in the include/socp.h layout (flat)."""
    B = len(c) // n
    P = params or Params()
    x, y, z, s = np.zeros(B * n), np.zeros(max(B * m, 1)), np.zeros(B * k), np.zeros(B * k)
    if warm is not None:
        x[:], z[:], s[:] = warm[0], warm[2], warm[3]
        if m:
            y[:] = warm[1]
        P = Params(P.maxit, P.tol, P.step, P.sigma_exp, P.init_eps, P.flags | F_WARM_START)
    iters, status = np.zeros(B, np.int32), np.zeros(B, np.int32)
    res = np.zeros(3 * B)
    if sing is None:  # the Problem constructor's rule (Socp.jl:49-56), per problem
        Gs = np.asarray(G, dtype=np.float64).reshape(B, k * n)
        sing = np.array([lib().or_sing(n, k, np.ascontiguousarray(Gs[p])) for p in range(B)], np.uint8)
    sg = np.ascontiguousarray(sing, dtype=np.uint8)
    rc = lib().or_batch_solve(B, n, m, k, *cone_arrays(cones), _f(c), _f(A) if m else np.zeros(1),
                              _f(b) if m else np.zeros(1), _f(G), _f(h),
                              sg.ctypes.data if sg is not None else None, C.byref(P),
                              x, y, z, s, iters, status, res.ctypes.data, nthreads)
    assert rc == 0
    return dict(x=x, y=y[:B * m], z=z, s=s, iters=iters, status=status, res=res.reshape(B, 3))


def generate(cones, B, n, m, k, seed, first_problem=0):
    """CPU restatement of socp_generate."""
    c, A, b = np.zeros(B * n), np.zeros(max(B * m * n, 1)), np.zeros(max(B * m, 1))
    G, h = np.zeros(B * k * n), np.zeros(B * k)
    lib().or_generate(B, n, m, k, *cone_arrays(cones), seed, first_problem, c, A, b, G, h)
    return dict(c=c, A=A[:B * m * n], b=b[:B * m], G=G, h=h)
