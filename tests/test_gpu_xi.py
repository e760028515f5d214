"""SOCP_F_EXPLICIT_INVERSE: the reference's operation order on the Cholesky shapes.

densesolver.jl:47-48 forms Li = H^-1 explicitly from the Cholesky factor
(ldiv!(Li, cholesky!(H), I)) and uses it in every solve (:73,83).  By default
the register kernel's m <= 16 shapes factor H = L L' and solve triangularly
instead; with the flag they form Li = L^-T L^-1 from the same tile factor
(chol_inv: Y = L^-1 by block forward substitution, Li = Y'Y), and S^-1 the
same way -- KM = 2 / 3 instantiations, so the default kernels are untouched.  Under the reference
stopping rule the two modes differ in OUTCOME on a pure LP:
with the explicit inverse chol(H) fails near the end of every solve, without
it every problem converges.  The explicit-inverse GPU run must reproduce the
reference-order oracle's outcomes and iteration counts there."""
import numpy as np
import pytest

import socp_amd as S
from socp_amd.configs import C1, C2

pytestmark = pytest.mark.gpu

LP = dict(n=32, m=8, k=48, cones=[(0, 0, 48)], seed=0x534F4350 + 9)


def rel(a, b):
    a, b = np.asarray(a).reshape(-1), np.asarray(b).reshape(-1)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def _lp(oracle, B):
    return oracle.generate(LP["cones"], B, LP["n"], LP["m"], LP["k"], LP["seed"])


def _gpu(d, cfg, B, **kw):
    return S.batch_solve(cfg["cones"], cfg["n"], cfg["m"], cfg["k"], d["c"], d["A"], d["b"], d["G"], d["h"],
                         np.zeros(B, np.uint8), **kw)


@pytest.mark.parametrize("force_large", [False, True])
def test_lp_reference_rule_matches_reference_order(oracle, force_large):
    """tol = 1e-5, maxit = 40 (solver.jl:105,122) on 256 pure LPs: the explicit
    -inverse kernel ends like the oracle in the reference's own op order (dense
    iW*iW', G'*iWiW*G, potrs(I)); the default kernel converges on all of them
    like the oracle's Cholesky-solve order."""
    B = 256
    d = _lp(oracle, B)
    n, m, k, cones = LP["n"], LP["m"], LP["k"], LP["cones"]
    sing = np.zeros(B, np.uint8)
    ref = oracle.batch_solve(cones, n, m, k, d["c"], d["A"], d["b"], d["G"], d["h"], sing=sing,
                             params=oracle.Params(maxit=40, tol=1e-5))
    chol = oracle.batch_solve(cones, n, m, k, d["c"], d["A"], d["b"], d["G"], d["h"], sing=sing,
                              params=oracle.Params(maxit=40, tol=1e-5, flags=oracle.F_STRUCTURED | oracle.F_CHOLSOLVE))
    xi = _gpu(d, LP, B, maxit=40, tol=1e-5, explicit_inverse=True, force_large=force_large)
    assert np.bincount(ref["status"], minlength=5)[2] == B  # the reference order: chol(H) fails on every LP
    same = xi["status"] == ref["status"]
    assert same.mean() >= 0.98, np.bincount(xi["status"], minlength=5)
    d_it = np.abs(xi["iters"] - ref["iters"])[same]
    assert (d_it <= 1).mean() >= 0.95, np.bincount(d_it)
    assert (d_it == 0).mean() >= 0.85, np.bincount(d_it)
    if not force_large:
        dflt = _gpu(d, LP, B, maxit=40, tol=1e-5)
        assert (chol["status"] == 0).all()
        assert (dflt["status"] == 0).mean() >= 0.99, np.bincount(dflt["status"], minlength=5)
        conv = (dflt["status"] == 0) & (chol["status"] == 0)
        assert (np.abs(dflt["iters"] - chol["iters"])[conv] <= 1).mean() >= 0.98


@pytest.mark.parametrize("cfg,maxk", [(C1, 3), (C2, 6)])
def test_explicit_inverse_trajectory(oracle, cfg, maxk):
    """P4 for the explicit-inverse kernel: fixed-K iterates vs the oracle's
    structured order (X = W^-1 G per cone, H = X'X, Li by potrs(I) -- the
    reference's inverse) and its Y'Y form (F_INV_YTY, the kernel's) rel <= 1e-8,
    and vs the reference order while the systems are well conditioned (first
    two iterations) rel <= 1e-8."""
    B = 16
    d = oracle.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    for K in range(1, maxk + 1):
        g = S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"],
                          np.zeros(B, np.uint8), maxit=K, tol=0.0, explicit_inverse=True)
        for flags, kmax in ((oracle.F_STRUCTURED, maxk), (oracle.F_STRUCTURED | oracle.F_INV_YTY, maxk), (0, 2)):
            if K > kmax:
                continue
            r = oracle.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"],
                                   params=oracle.Params(maxit=K, tol=0.0, flags=flags))
            assert (g["status"] == r["status"]).all()
            for p in range(B):
                for key, L in (("x", cfg.n), ("z", cfg.k), ("s", cfg.k)):
                    e = rel(g[key][p * L:(p + 1) * L], r[key][p * L:(p + 1) * L])
                    assert e <= 1e-8, (flags, K, p, key, e)


def test_explicit_inverse_kkt_golden_and_split(kats):
    """P2 (runtests.jl:95-128 golden) through the explicit-inverse entries, and
    the split plugin (socp_dense_*) bitwise equal to the fused entry."""
    g = kats["kkt_golden"]
    cones = [tuple(c) for c in g["cones"]]
    G = np.array(g["G"]).ravel(order="F")
    args = (np.array(g["s"]), np.array(g["z"]), np.array(g["dx"]), None, np.array(g["dz"]), np.array(g["ds"]))
    out = S.batch_kkt_solve(cones, 3, 0, 4, None, G, None, *args, explicit_inverse=True)
    assert out["status"][0] == 0
    for key in ("cx", "cz", "cs"):
        assert np.abs(out[key] - np.array(g[key])).max() <= 1e-10, key
    h = S.DenseHandle(cones, 3, 0, 4, None, G, None, explicit_inverse=True)
    assert (h.setup_iter(args[0], args[1]) == 0).all()
    r = h.solve_kkt(args[2], args[3], args[4], args[5])
    for key in ("cx", "cz", "cs"):
        assert np.array_equal(r[key], out[key]), key
    h.close()


def test_explicit_inverse_split_equals_fused_c2(oracle):
    """C2 batch at an interior iterate: socp_dense_* with the flag = the fused
    explicit-inverse entry bitwise; both within 1e-9 of the default (Cholesky)
    kernel's solve, which is the same linear system."""
    cfg, B = C2, 64
    d = oracle.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    it = S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"],
                       np.zeros(B, np.uint8), maxit=2, tol=0.0)
    rng = np.random.default_rng(3)
    rhs = [rng.standard_normal(B * q) for q in (cfg.n, cfg.m, cfg.k, cfg.k)]
    fused = S.batch_kkt_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["A"], d["G"], np.zeros(B, np.uint8), it["s"], it["z"],
                              *rhs, explicit_inverse=True)
    dflt = S.batch_kkt_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["A"], d["G"], np.zeros(B, np.uint8), it["s"], it["z"],
                             *rhs)
    h = S.DenseHandle(cfg.cones, cfg.n, cfg.m, cfg.k, d["A"], d["G"], np.zeros(B, np.uint8), explicit_inverse=True)
    assert (h.setup_iter(it["s"], it["z"]) == 0).all()
    split = h.solve_kkt(*rhs)
    h.close()
    assert (fused["status"] == 0).all()
    for key in ("cx", "cy", "cz", "cs"):
        assert np.array_equal(split[key], fused[key]), key
        assert rel(fused[key], dflt[key]) <= 1e-9, (key, rel(fused[key], dflt[key]))


@pytest.mark.parametrize("cfg", [C1, C2], ids=["C1", "C2"])
def test_explicit_inverse_trajectory_at_its_rounding_floor(oracle, cfg):
    """The explicit-inverse kernel through the bench K against the oracle in its
    own operation order (X = W^-1 G, Li = Y'Y with Y = L^-1: F_STRUCTURED |
    F_INV_YTY), gated by the oracle's sensitivity to one rounding:
    rel <= 10 floor_K + 1e-13 for every K, vector and problem (8 problems)."""
    from problems import trajectory_at_floor
    B = 8
    d = oracle.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    rows = trajectory_at_floor(
        oracle, cfg, d, B, cfg.fixed_k, oracle.F_STRUCTURED | oracle.F_INV_YTY,
        lambda K: S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"],
                                np.zeros(B, np.uint8), maxit=K, tol=0.0, explicit_inverse=True))
    print("worst error / gate (ratio, K, problem, vector, error, floor):", rows[:4])
    assert rows[0][0] <= 1.0, rows[:6]
