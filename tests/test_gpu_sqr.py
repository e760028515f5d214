"""The rank-update plugin (socp_sqr_*): SqrScaling + SparseSolver
(sqrscalings.jl:8-214, spsolver.jl:1-130) on the GPU.

Gates (fp64; CHOLMOD's permutation and supernodal order are replaced by a
dense factor, so agreement is to rounding, never bitwise):
  * the reference's KKT golden (runtests.jl:95-128 -- produced on exactly this
    path) through the HIP plugin <= 1e-10;
  * the factor after modify_factors! inverts to the dense H^-1
    (runtests.jl:62-77) <= 1e-10, and l, wbs, mu equal the dense scaling's
    (runtests.jl:58-60, 71-73);
  * batches at the C1/C2 shapes at interior iterates: HIP vs the oracle's
    rank-update restatement, rel <= 1e-9 where kappa(H) <= 1e5; HIP sqr vs the
    HIP dense plugin at the same tolerance; m = 0 and sing problems;
  * every instantiation (NC = 16, 32, 48, 64) and the shape limits (m = 64,
    15 cones, k = 1000 on one wavefront, n = 1000 / m = 300 on the workgroup
    kernels, an LP with no SOC cone) vs the oracle, gate
    max(1e-9, 1e-15 kappa(H) kappa(S));
  * failures (domain error, lost definiteness in a downdate) stay in their
    problem; solve_kkt before setup_iter is refused; per-call H2D bytes.
"""
import numpy as np
import pytest

import socp_amd as S
from socp_amd.configs import C1, C2

pytestmark = pytest.mark.gpu


def iterates(oracle, cfg, B, K):
    d = oracle.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    r = oracle.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"],
                           sing=np.zeros(B, np.uint8), params=oracle.Params(maxit=K, tol=0.0))
    return dict(A=d["A"], G=d["G"], s=r["s"], z=r["z"])


def rhs(cfg, B, seed):
    rng = np.random.default_rng(seed)
    return [rng.standard_normal(B * q) for q in (cfg.n, cfg.m, cfg.k, cfg.k)]


def per_problem(v, B):
    return v.reshape(B, -1)


def test_sqr_kkt_golden_through_hip(kats):
    g = kats["kkt_golden"]
    cones = [tuple(c) for c in g["cones"]]
    G = np.array(g["G"], dtype=np.float64)
    k, n = G.shape
    h = S.SqrHandle(cones, n, 0, k, None, G.ravel(order="F"))
    st = h.setup_iter(np.array(g["s"]), np.array(g["z"]))
    assert st[0] == 0
    out = h.solve_kkt(np.array(g["dx"]), None, np.array(g["dz"]), np.array(g["ds"]))
    assert out["status"][0] == 0
    for key in ("cx", "cz", "cs"):
        assert np.abs(out[key] - np.array(g[key])).max() < 1e-10, key


def test_sqr_kkt_golden_through_mirror(kats):
    # the reference's own call sequence: SparseSolver(prob), setup_iter, solve_kkt
    g = kats["kkt_golden"]
    cones = [S.POC(0, 1), S.SOC(1, 3)]
    prob = S.Problem([-1.0, -1.0, 1.0], np.zeros((0, 3)), np.zeros(0), np.array(g["G"]), [5.0, 0, 0, 0], cones)
    solver = S.SparseSolver(prob)
    state = S.State(prob, np.zeros(3), np.zeros(0), g["z"], g["s"])
    sc = S.compute_scaling(prob.cones, S.SqrScaling(prob), state.s, state.z)
    S.setup_iter(solver, prob, state, sc)
    cx, cy, cz, cs = np.zeros(3), np.zeros(0), np.zeros(4), np.zeros(4)
    S.solve_kkt(solver, prob, state, sc, np.array(g["dx"]), np.zeros(0), np.array(g["dz"]), np.array(g["ds"]),
                cx, cy, cz, cs)
    for key, v in (("cx", cx), ("cz", cz), ("cs", cs)):
        assert np.abs(v - np.array(g[key])).max() < 1e-10, key
    assert np.all(sc.l > 0) and sc.mu[1] > 0


def test_sqr_factor_and_scaling_match_dense(kats, oracle):
    q = kats["sqr_scaling"]
    cones = [tuple(c) for c in q["cones"]]
    G = np.array(q["G"], dtype=np.float64)
    k, n = G.shape
    pairs = q["pairs"]
    B = len(pairs)
    s = np.concatenate([p["s"] for p in pairs])
    z = np.concatenate([p["z"] for p in pairs])
    h = S.SqrHandle(cones, n, 0, k, None, np.tile(G.ravel(order="F"), B))
    assert (h.setup_iter(s, z) == 0).all()
    sc_dev = h.scaling()
    for p, pair in enumerate(pairs):
        sc = oracle.compute_scaling(cones, np.array(pair["s"]), np.array(pair["z"]))
        L = h.factor(p)
        assert np.abs(np.triu(L, 1)).max() == 0.0
        Hd = G.T @ sc["iWiW"] @ G
        assert np.abs(np.linalg.inv(L @ L.T) - np.linalg.inv(Hd)).max() < 1e-10
        assert np.abs(sc_dev["l"][p] - sc["l"]).max() < 1e-12
        assert np.abs(sc_dev["wbs"][p] - sc["wbs"]).max() < 1e-12
        assert abs(sc_dev["mu"][p][1] - sc["mu"][1]) < 1e-12


@pytest.mark.parametrize("cfg,K", [(C1, 2), (C2, 3), (C2, 6)])
def test_sqr_batch_matches_oracle(oracle, cfg, K):
    B = 64
    it = iterates(oracle, cfg, B, K)
    h = S.SqrHandle(cfg.cones, cfg.n, cfg.m, cfg.k, it["A"], it["G"], np.zeros(B, np.uint8))
    st = h.setup_iter(it["s"], it["z"])
    r = rhs(cfg, B, 7)
    got = h.solve_kkt(*r)
    dense = S.DenseHandle(cfg.cones, cfg.n, cfg.m, cfg.k, it["A"], it["G"], np.zeros(B, np.uint8))
    dst = dense.setup_iter(it["s"], it["z"])
    dref = dense.solve_kkt(*r)
    n, m, k = cfg.n, cfg.m, cfg.k
    checked = 0
    for p in range(B):
        A = it["A"][p * m * n:(p + 1) * m * n].reshape(n, m).T
        G = it["G"][p * k * n:(p + 1) * k * n].reshape(n, k).T
        sl = lambda v, q: v[p * q:(p + 1) * q]  # noqa: E731
        o = oracle.sqr_kkt_single(cfg.cones, A, G, False, sl(it["s"], k), sl(it["z"], k), sl(r[0], n), sl(r[1], m),
                                  sl(r[2], k), sl(r[3], k))
        assert st[p] == o["status"] == dst[p], p
        if o["status"]:
            continue
        L = o["L"]
        kappa = np.linalg.cond(L @ L.T)
        if kappa > 1e5:
            continue
        checked += 1
        for key, q in (("cx", n), ("cy", m), ("cz", k), ("cs", k)):
            ref = o[key]
            scale = max(np.abs(ref).max(), 1e-300)
            assert np.abs(sl(got[key], q) - ref).max() <= 1e-9 * scale, (p, key)
            assert np.abs(sl(got[key], q) - sl(dref[key], q)).max() <= 1e-9 * scale, (p, key, "vs dense")
    assert checked >= B // 2


def test_sqr_m0_and_sing(oracle):
    """m = 0 (no equality rows) and a sing problem (G'G singular: the A'A term
    enters H, spsolver.jl:66-71; the sing branch m0 = dy - cy, :115-118)."""
    rng = np.random.default_rng(3)
    cones = [(0, 0, 4), (1, 4, 6)]
    n, k = 6, 10
    for m, sing in ((0, False), (3, True)):
        B = 8
        G = rng.standard_normal((B, k, n))
        if sing:
            G[:, :, -1] = 0.0  # last column unused by the cones: G'G singular
        A = rng.standard_normal((B, m, n))
        s = np.zeros((B, k))
        z = np.zeros((B, k))
        for arr in (s, z):
            arr[:, :4] = rng.uniform(0.5, 2.0, (B, 4))
            arr[:, 5:] = rng.uniform(-0.3, 0.3, (B, 5))
            arr[:, 4] = np.linalg.norm(arr[:, 5:], axis=1) + rng.uniform(0.2, 1.0, B)
        Gf = np.concatenate([G[p].ravel(order="F") for p in range(B)])
        Af = np.concatenate([A[p].ravel(order="F") for p in range(B)]) if m else None
        singv = np.full(B, 1 if sing else 0, np.uint8)
        h = S.SqrHandle(cones, n, m, k, Af, Gf, singv)
        assert (h.setup_iter(s.ravel(), z.ravel()) == 0).all()
        r = [rng.standard_normal(B * q) for q in (n, m, k, k)]
        got = h.solve_kkt(r[0], r[1] if m else None, r[2], r[3])
        for p in range(B):
            sl = lambda v, q: v[p * q:(p + 1) * q]  # noqa: E731
            o = oracle.sqr_kkt_single(cones, A[p], G[p], sing, s[p], z[p], sl(r[0], n), sl(r[1], m), sl(r[2], k),
                                      sl(r[3], k))
            assert o["status"] == 0
            for key, q in (("cx", n), ("cy", m), ("cz", k), ("cs", k)):
                if q == 0:
                    continue
                assert np.abs(sl(got[key], q) - o[key]).max() <= 1e-9 * max(1.0, np.abs(o[key]).max()), (m, p, key)


def test_sqr_failures_are_isolated(oracle):
    cfg, B = C2, 16
    it = iterates(oracle, cfg, B, 2)
    s, z = it["s"].copy(), it["z"].copy()
    k = cfg.k
    s[3 * k + 40] = -50.0                 # problem 3: s outside its SOC -> sqrt of a negative (DomainError)
    z[5 * k + 2] = -1.0                   # problem 5: POC z < 0 -> z/s < 0 -> DomainError
    h = S.SqrHandle(cfg.cones, cfg.n, cfg.m, cfg.k, it["A"], it["G"], np.zeros(B, np.uint8))
    st = h.setup_iter(s, z)
    assert st[3] == S.DOMAIN_ERROR and st[5] == S.DOMAIN_ERROR
    good = [p for p in range(B) if p not in (3, 5)]
    assert (st[good] == 0).all()
    r = rhs(cfg, B, 1)
    out = h.solve_kkt(*r)
    assert out["status"][3] == S.DOMAIN_ERROR
    assert np.isnan(out["cx"][3 * cfg.n:4 * cfg.n]).all()
    clean = S.SqrHandle(cfg.cones, cfg.n, cfg.m, cfg.k, it["A"], it["G"], np.zeros(B, np.uint8))
    clean.setup_iter(it["s"], it["z"])
    ref = clean.solve_kkt(*r)
    for p in good:  # neighbours are untouched, bit for bit
        assert np.array_equal(out["cx"][p * cfg.n:(p + 1) * cfg.n], ref["cx"][p * cfg.n:(p + 1) * cfg.n])


def test_sqr_refuses_solve_before_setup_and_counts_bytes(oracle):
    cfg, B = C1, 8
    it = iterates(oracle, cfg, B, 1)
    h = S.SqrHandle(cfg.cones, cfg.n, cfg.m, cfg.k, it["A"], it["G"], np.zeros(B, np.uint8))
    with pytest.raises(S.SocpError):
        h.solve_kkt(*rhs(cfg, B, 0))
    h.setup_iter(it["s"], it["z"])
    assert h.h2d_bytes == B * 2 * cfg.k * 8
    h.solve_kkt(*rhs(cfg, B, 0))
    assert h.h2d_bytes == B * (cfg.n + cfg.m + 2 * cfg.k) * 8
    assert h.record_bytes >= (cfg.n * cfg.n + cfg.m * cfg.m + 2 * cfg.k) * 8


def test_sqr_device_tensors_equal_host():
    import torch
    cfg, B = C2, 32
    d = S.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    c, A, b, G, hh = d
    out = S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, c, A, b, G, hh, torch.zeros(B, dtype=torch.uint8,
                        device=G.device), maxit=3, tol=0.0)
    S.default_context().sync()
    s, z = out["s"], out["z"]
    hd = S.SqrHandle(cfg.cones, cfg.n, cfg.m, cfg.k, A, G, torch.zeros(B, dtype=torch.uint8, device=G.device))
    hh_ = S.SqrHandle(cfg.cones, cfg.n, cfg.m, cfg.k, A.cpu().numpy(), G.cpu().numpy(), np.zeros(B, np.uint8))
    std = hd.setup_iter(s, z)
    sth = hh_.setup_iter(s.cpu().numpy(), z.cpu().numpy())
    r = rhs(cfg, B, 4)
    od = hd.solve_kkt(*[torch.from_numpy(v).to(G.device) for v in r])
    torch.cuda.synchronize()
    oh = hh_.solve_kkt(*r)
    assert np.array_equal(std.cpu().numpy(), sth)
    for key in ("cx", "cy", "cz", "cs"):
        assert np.array_equal(od[key].cpu().numpy(), oh[key]), key


def _interior(rng, cones, B, k):
    """B interior points of the cone product (POC entries > 0, SOC heads above the tail norm)."""
    v = np.zeros((B, k))
    for kind, o, d in cones:
        if kind == 0:
            v[:, o:o + d] = rng.uniform(0.3, 2.0, (B, d))
        else:
            v[:, o + 1:o + d] = rng.uniform(-0.4, 0.4, (B, d - 1))
            v[:, o] = np.linalg.norm(v[:, o + 1:o + d], axis=1) + rng.uniform(0.2, 1.0, B)
    return v


@pytest.mark.parametrize("n,m,k,cones", [
    (40, 8, 60, [(0, 0, 20), (1, 20, 40)]),                     # NC = 48
    (17, 3, 25, [(1, 0, 5), (1, 5, 9), (1, 14, 11)]),            # NC = 32, ragged, three SOC cones
    (64, 64, 100, [(0, 0, 36), (1, 36, 64)]),                    # m at its limit, k > 64
    (9, 0, 12, [(0, 0, 12)]),                                    # LP: no SOC cone, no modification
    (30, 5, 256, [(0, 0, 16)] + [(1, 16 + 16 * i, 16) for i in range(15)]),  # 15 cones
    (30, 5, 1000, [(0, 0, 100)] + [(1, 100 + 75 * i, 75) for i in range(12)]),  # one wavefront, k > 256
])
def test_sqr_shapes_vs_oracle(oracle, n, m, k, cones):
    rng = np.random.default_rng(n * 1000 + m * 10 + k)
    B = 12
    G = rng.standard_normal((B, k, n))
    A = rng.standard_normal((B, m, n))
    s, z = _interior(rng, cones, B, k), _interior(rng, cones, B, k)
    Gf = np.concatenate([G[p].ravel(order="F") for p in range(B)])
    Af = np.concatenate([A[p].ravel(order="F") for p in range(B)]) if m else None
    h = S.SqrHandle(cones, n, m, k, Af, Gf, np.zeros(B, np.uint8))
    st = h.setup_iter(s.ravel(), z.ravel())
    r = [rng.standard_normal(B * q) for q in (n, m, k, k)]
    got = h.solve_kkt(r[0], r[1] if m else None, r[2], r[3])
    for p in range(B):
        sl = lambda v, q: v[p * q:(p + 1) * q]  # noqa: E731
        o = oracle.sqr_kkt_single(cones, A[p], G[p], False, s[p], z[p], sl(r[0], n), sl(r[1], m), sl(r[2], k),
                                  sl(r[3], k))
        assert st[p] == o["status"], p
        if o["status"]:
            continue
        assert np.abs(np.tril(h.factor(p)) - o["L"]).max() <= 1e-9 * np.abs(o["L"]).max(), p
        # rounding-level agreement, scaled by the conditioning of H and S = A H^-1 A'
        Hm = o["L"] @ o["L"].T
        kap = np.linalg.cond(Hm) * (np.linalg.cond(A[p] @ np.linalg.solve(Hm, A[p].T)) if m else 1.0)
        tol = max(1e-9, 1e-15 * kap)
        for key, q in (("cx", n), ("cy", m), ("cz", k), ("cs", k)):
            if q:
                ref = o[key]
                assert np.abs(sl(got[key], q) - ref).max() <= tol * max(1.0, np.abs(ref).max()), (p, key, kap)


def test_sqr_optimal_control_n150(oracle):
    """The reference's own sparse-path problem (runtests.jl:204-244 'linear
    optimal control', timed there on SparseSolver): n=150, m=102, k=50, one
    SOC(50), G'G singular (sing: H = G'W^-2G + A'A).  Past the wavefront
    kernels, so the workgroup kernels (factor packed in LDS) run it; iterates
    of the oracle's rank-update IPM (F_SQR) at K = 1..4."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from problems import optimal_control
    cones, c, A, b, G, h = optimal_control(50)
    n, m, k = len(c), A.shape[0], G.shape[0]
    assert oracle.sing_flag(G)
    rng = np.random.default_rng(150)
    for K in (1, 2, 3, 4):
        tr = oracle.solve_trace(cones, c, A, b, G, h, params=oracle.Params(maxit=K, tol=0.0, flags=oracle.F_SQR))
        s, z = np.asarray(tr["s"]), np.asarray(tr["z"])
        hd = S.SqrHandle(cones, n, m, k, A.ravel(order="F"), G.ravel(order="F"), np.ones(1, np.uint8))
        st = hd.setup_iter(s, z)
        r = [rng.standard_normal(q) for q in (n, m, k, k)]
        got = hd.solve_kkt(*r)
        o = oracle.sqr_kkt_single(cones, A, G, True, s, z, *r)
        assert st[0] == o["status"] == 0, (K, st[0], o["status"])
        assert S.default_context().last_kernel_name() == "socp_sqr_solve_wg_kernel"
        assert np.abs(np.tril(hd.factor(0)) - o["L"]).max() <= 1e-9 * np.abs(o["L"]).max(), K
        Hm = o["L"] @ o["L"].T
        kap = np.linalg.cond(Hm) * np.linalg.cond(A @ np.linalg.solve(Hm, A.T))
        tol = max(1e-9, 1e-15 * kap)
        for key in ("cx", "cy", "cz", "cs"):
            ref = o[key]
            assert np.abs(got[key] - ref).max() <= tol * max(1.0, np.abs(ref).max()), (K, key, kap)


@pytest.mark.parametrize("n,m,k,cones,sing", [
    (100, 30, 120, [(0, 0, 40), (1, 40, 80)], False),               # n > 64
    (70, 66, 100, [(1, 0, 50), (1, 50, 50)], True),                 # m > 64: sing, A'A in H
    (160, 160, 256, [(0, 0, 16)] + [(1, 16 + 16 * i, 16) for i in range(15)], True),  # n, m, k at their limits
    (77, 0, 90, [(1, 0, 30), (1, 30, 29), (1, 59, 31)], False),     # ragged SOC cones, m = 0
    (129, 65, 140, [(0, 0, 140)], False),                           # LP: no modification, odd sizes
    # beyond the LDS-packed factor (SqrLayout::gfac: the packed factors and the
    # C chunk in the record)
    (300, 120, 400, [(0, 0, 100)] + [(1, 100 * i, 100) for i in range(1, 4)], False),
    (520, 200, 600, [(1, 0, 300), (1, 300, 300)], False),
    (256, 256, 300, [(1, 0, 150), (1, 150, 150)], True),            # sing, m = n
    # near the advertised limits (n, m <= 1024): factors and C in the record,
    # m > 256 (the two-pass residual form's range)
    (1000, 300, 1100, [(0, 0, 100)] + [(1, 100 + 200 * i, 200) for i in range(5)], False),
])
def test_sqr_workgroup_shapes_vs_oracle(oracle, n, m, k, cones, sing):
    rng = np.random.default_rng(n * 1000 + m * 10 + k)
    B = 6
    G = rng.standard_normal((B, k, n))
    if sing:
        G[:, :, n // 2:] = 0.0  # G'G singular: the A'A term carries H
    A = rng.standard_normal((B, m, n))
    s, z = _interior(rng, cones, B, k), _interior(rng, cones, B, k)
    Gf = np.concatenate([G[p].ravel(order="F") for p in range(B)])
    Af = np.concatenate([A[p].ravel(order="F") for p in range(B)]) if m else None
    h = S.SqrHandle(cones, n, m, k, Af, Gf, np.full(B, 1 if sing else 0, np.uint8))
    st = h.setup_iter(s.ravel(), z.ravel())
    r = [rng.standard_normal(B * q) for q in (n, m, k, k)]
    got = h.solve_kkt(r[0], r[1] if m else None, r[2], r[3])
    assert S.default_context().last_kernel_name() == "socp_sqr_solve_wg_kernel"
    ok = 0
    for p in range(B):
        sl = lambda v, q: v[p * q:(p + 1) * q]  # noqa: E731
        o = oracle.sqr_kkt_single(cones, A[p], G[p], sing, s[p], z[p], sl(r[0], n), sl(r[1], m), sl(r[2], k),
                                  sl(r[3], k))
        assert st[p] == o["status"], p
        if o["status"]:
            assert np.isnan(sl(got["cx"], n)).all()
            continue
        ok += 1
        assert np.abs(np.tril(h.factor(p)) - o["L"]).max() <= 1e-9 * np.abs(o["L"]).max(), p
        Hm = o["L"] @ o["L"].T
        kap = np.linalg.cond(Hm) * (np.linalg.cond(A[p] @ np.linalg.solve(Hm, A[p].T)) if m else 1.0)
        tol = max(1e-9, 1e-15 * kap)
        for key, q in (("cx", n), ("cy", m), ("cz", k), ("cs", k)):
            if q:
                ref = o[key]
                assert np.abs(sl(got[key], q) - ref).max() <= tol * max(1.0, np.abs(ref).max()), (p, key, kap)
    assert ok >= B // 2


def test_sqr_solve_socp_large_shape(oracle):
    """solve_socp on the rank-update plugin beyond the old n, m <= 160, k <= 256
    cap (the record-resident factors, the IPM's two-pass residuals for k > 256):
    fixed-K trajectories vs the oracle's F_SQR IPM, rel <= 1e-8."""
    n, m, k = 300, 40, 360
    cones = [(0, 0, 60)] + [(1, 60 + 100 * i, 100) for i in range(3)]
    B = 2
    d = oracle.generate(cones, B, n, m, k, 0x534F4350 + 21)
    for K in (1, 2):
        r = oracle.batch_solve(cones, n, m, k, d["c"], d["A"], d["b"], d["G"], d["h"], sing=np.zeros(B, np.uint8),
                               params=oracle.Params(maxit=K, tol=0.0, flags=oracle.F_SQR))
        hd = S.SqrHandle(cones, n, m, k, d["A"], d["G"], np.zeros(B, np.uint8))
        g = hd.solve_socp(d["c"], d["b"], d["h"], maxit=K, tol=0.0)
        assert (g["status"] == r["status"]).all() and (g["iters"] == r["iters"]).all()
        for p in range(B):
            for key, L in (("x", n), ("z", k), ("s", k)):
                a_, b_ = g[key][p * L:(p + 1) * L], r[key][p * L:(p + 1) * L]
                e = np.linalg.norm(a_ - b_) / np.linalg.norm(b_)
                assert e <= 1e-8, (K, p, key, e)


def test_sqr_solve_socp_wide_k_dynamic_lds(oracle):
    """solve_socp with k = 1500 on the one-wavefront plugin kernels: the IPM
    kernels' vectors ((7k + 64) doubles = 84 KB) pass the default 64 KiB of
    dynamic LDS, so every IPM kernel opts in (hipFuncSetAttribute).  Fixed-K
    trajectories vs the oracle's F_SQR IPM, rel <= 1e-8."""
    n, m, k = 40, 10, 1500
    cones = [(0, 0, 300)] + [(1, 300 + 100 * i, 100) for i in range(12)]
    B = 3
    d = oracle.generate(cones, B, n, m, k, 0x534F4350 + 22)
    for K in (1, 3):
        r = oracle.batch_solve(cones, n, m, k, d["c"], d["A"], d["b"], d["G"], d["h"], sing=np.zeros(B, np.uint8),
                               params=oracle.Params(maxit=K, tol=0.0, flags=oracle.F_SQR))
        hd = S.SqrHandle(cones, n, m, k, d["A"], d["G"], np.zeros(B, np.uint8))
        g = hd.solve_socp(d["c"], d["b"], d["h"], maxit=K, tol=0.0)
        assert (g["status"] == r["status"]).all() and (g["iters"] == r["iters"]).all()
        for p in range(B):
            for key, L in (("x", n), ("z", k), ("s", k)):
                a_, b_ = g[key][p * L:(p + 1) * L], r[key][p * L:(p + 1) * L]
                e = np.linalg.norm(a_ - b_) / np.linalg.norm(b_)
                assert e <= 1e-8, (K, p, key, e)


def test_sqr_workgroup_failures_isolated(oracle):
    """A domain error and a lost downdate in one problem of a workgroup-kernel
    batch leave its neighbours bit-identical."""
    rng = np.random.default_rng(11)
    n, m, k, B = 90, 20, 100, 5
    cones = [(0, 0, 20), (1, 20, 80)]
    G = rng.standard_normal((B, k, n))
    A = rng.standard_normal((B, m, n))
    s, z = _interior(rng, cones, B, k), _interior(rng, cones, B, k)
    Gf = np.concatenate([G[p].ravel(order="F") for p in range(B)])
    Af = np.concatenate([A[p].ravel(order="F") for p in range(B)])
    r = [rng.standard_normal(B * q) for q in (n, m, k, k)]
    clean = S.SqrHandle(cones, n, m, k, Af, Gf, np.zeros(B, np.uint8))
    assert (clean.setup_iter(s.ravel(), z.ravel()) == 0).all()
    ref = clean.solve_kkt(*r)
    s2 = s.copy()
    s2[2, 30] = 50.0  # problem 2: SOC tail above its head -> sqrt of a negative
    bad = S.SqrHandle(cones, n, m, k, Af, Gf, np.zeros(B, np.uint8))
    st = bad.setup_iter(s2.ravel(), z.ravel())
    assert st[2] == S.DOMAIN_ERROR and (st[[0, 1, 3, 4]] == 0).all()
    out = bad.solve_kkt(*r)
    assert np.isnan(out["cx"][2 * n:3 * n]).all()
    for p in (0, 1, 3, 4):
        assert np.array_equal(out["cx"][p * n:(p + 1) * n], ref["cx"][p * n:(p + 1) * n])


# ---------------------------------------------------------------- solve_socp
# solve_socp(prob, SolverState(prob, SparseSolver(prob))) -- the reference's own
# tested configuration (runtests.jl:143-144, 188-189) -- batched on the device
# (socp_sqr_solve_socp).  The oracle's F_SQR mode restates the same algorithm
# (sqrscalings.jl / spsolver.jl in the solver.jl loop).

@pytest.mark.parametrize("name", ["soc1", "soc2", "soc3"])
def test_sqr_solve_socp_runtests_kats(kats, oracle, name):
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from problems import kat_problem
    q = kats[name]
    cones, c, A, b, G, h = kat_problem(q)
    prob = S.Problem(c, A, b, G, h, cones)
    ss = S.SolverState(prob, S.SparseSolver(prob))
    st = S.solve_socp(prob, ss)
    assert ss.status == S.CONVERGED
    assert np.linalg.norm(st.x - np.array(q["x_expect"])) < q["tol"]  # runtests.jl's own assertion
    r = oracle.solve_trace(cones, c, A, b, G, h, params=oracle.Params(flags=oracle.F_SQR))
    assert r["status"] == 0
    assert abs(ss.iters - r["iters"]) <= 1
    assert np.abs(st.x - r["x"]).max() <= 1e-3


@pytest.mark.parametrize("cfg,K", [(C1, 3), (C2, 4), (C2, 6)])
def test_sqr_solve_socp_trajectory(oracle, cfg, K):
    """Fixed-K solves (tol = 0) from the same start: the HIP rank-update IPM
    against the oracle's F_SQR IPM, relative error of x, z, s <= 1e-8 (SURVEY
    §8(c) P4's gate; the W = I initial solve and the oracle's LU initial solve
    agree to rounding)."""
    B = 32
    d = oracle.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    r = oracle.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"],
                           sing=np.zeros(B, np.uint8), params=oracle.Params(maxit=K, tol=0.0, flags=oracle.F_SQR))
    hd = S.SqrHandle(cfg.cones, cfg.n, cfg.m, cfg.k, d["A"], d["G"], np.zeros(B, np.uint8))
    g = hd.solve_socp(d["c"], d["b"], d["h"], maxit=K, tol=0.0)
    assert S.default_context().last_kernel_name() == "socp_sqr_solve_socp"
    assert (g["status"] == r["status"]).all()
    assert (g["iters"] == r["iters"]).all()
    for p in range(B):
        for key, L in (("x", cfg.n), ("z", cfg.k), ("s", cfg.k)):
            a_, b_ = g[key][p * L:(p + 1) * L], r[key][p * L:(p + 1) * L]
            e = np.linalg.norm(a_ - b_) / np.linalg.norm(b_)
            assert e <= 1e-8, (p, key, e)


@pytest.mark.parametrize("case", ["sing", "m0"])
def test_sqr_solve_socp_trajectory_sing_and_m0(oracle, case):
    """The wave kernels' whole-IPM path (the setup kernel's fused residuals,
    SqrArgs::fuse_resid) with `sing` problems (H = G'DG + A'A, m0 = dy - cy;
    every other problem of the batch) and with no equality constraints (m = 0):
    fixed-K trajectories vs the oracle's F_SQR IPM, rel <= 1e-8, equal status
    and iteration counts."""
    cfg, B, K = C1, 16, 3
    m = 0 if case == "m0" else cfg.m
    d = oracle.generate(cfg.cones, B, cfg.n, m, cfg.k, cfg.seed + 7)
    sing = (np.arange(B) % 2).astype(np.uint8) if case == "sing" else np.zeros(B, np.uint8)
    r = oracle.batch_solve(cfg.cones, cfg.n, m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"], sing=sing,
                           params=oracle.Params(maxit=K, tol=0.0, flags=oracle.F_SQR))
    hd = S.SqrHandle(cfg.cones, cfg.n, m, cfg.k, d["A"], d["G"], sing)
    g = hd.solve_socp(d["c"], d["b"], d["h"], maxit=K, tol=0.0)
    assert (g["status"] == r["status"]).all() and (g["iters"] == r["iters"]).all()
    for p in range(B):
        for key, L in (("x", cfg.n), ("z", cfg.k), ("s", cfg.k)):
            a_, b_ = g[key][p * L:(p + 1) * L], r[key][p * L:(p + 1) * L]
            e = np.linalg.norm(a_ - b_) / np.linalg.norm(b_)
            assert e <= 1e-8, (p, key, e)


def test_sqr_solve_socp_reference_rule_outcomes(oracle):
    """The reference stopping rule (tol = 1e-5 absolute, maxit = 40) on 256 C2
    problems: outcome statistics of the HIP rank-update IPM vs the oracle's
    F_SQR IPM (late iterations are decided at rounding level, SURVEY §0.7, so
    the gates are statistical, as for the dense path)."""
    cfg, B = C2, 256
    d = oracle.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    r = oracle.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"],
                           sing=np.zeros(B, np.uint8), params=oracle.Params(flags=oracle.F_SQR))
    hd = S.SqrHandle(cfg.cones, cfg.n, cfg.m, cfg.k, d["A"], d["G"], np.zeros(B, np.uint8))
    g = hd.solve_socp(d["c"], d["b"], d["h"])
    hg = np.bincount(g["status"], minlength=5)
    hr = np.bincount(r["status"], minlength=5)
    print("HIP", hg.tolist(), "oracle", hr.tolist())
    conv = (g["status"] == 0) & (r["status"] == 0)
    oc = r["status"] == 0
    assert hg[0] >= hr[0] - 0.03 * B, (hg, hr)
    assert conv.sum() >= 0.9 * oc.sum(), (conv.sum(), oc.sum())
    assert (np.abs(g["iters"][conv] - r["iters"][conv]) <= 1).mean() >= 0.95
    # converged problems satisfy the exit test at the returned iterate
    res = g["res"].reshape(B, 3)
    assert (res[g["status"] == 0].sum(axis=1) < 1e-5).all()
    dx = np.abs(g["x"].reshape(B, -1) - r["x"].reshape(B, -1)).max(axis=1)
    assert np.median(dx[conv]) <= 1e-3


def test_sqr_solve_socp_optimal_control_n150(oracle):
    """runtests.jl:204-244, the problem the reference times on SparseSolver:
    end to end on the workgroup kernels (n = 150, m = 102, sing)."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from problems import optimal_control
    cones, c, A, b, G, h = optimal_control(50)
    prob = S.Problem(c, A, b, G, h, cones)
    assert prob.sing
    ss = S.SolverState(prob, S.SparseSolver(prob))
    st = S.solve_socp(prob, ss)
    r = oracle.solve_trace(cones, c, A, b, G, h, params=oracle.Params(flags=oracle.F_SQR))
    assert ss.status == r["status"] == 0, (ss.status, r["status"])
    assert abs(ss.iters - r["iters"]) <= 1
    assert np.abs(st.x - r["x"]).max() <= 1e-3 * max(1.0, np.abs(r["x"]).max())


def test_sqr_solve_socp_isolation_and_device(oracle):
    """One problem broken (NaN in its h) stops alone -- its neighbours are
    bit-identical to a clean batch; device tensors give the host results bit
    for bit."""
    import torch
    cfg, B = C1, 16
    d = oracle.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    hd = S.SqrHandle(cfg.cones, cfg.n, cfg.m, cfg.k, d["A"], d["G"], np.zeros(B, np.uint8))
    clean = hd.solve_socp(d["c"], d["b"], d["h"])
    hbad = d["h"].copy()
    hbad[5 * cfg.k + 3] = np.nan
    bad = hd.solve_socp(d["c"], d["b"], hbad)
    assert bad["status"][5] != 0
    for p in range(B):
        if p == 5:
            continue
        assert bad["status"][p] == clean["status"][p] and bad["iters"][p] == clean["iters"][p]
        assert np.array_equal(bad["x"][p * cfg.n:(p + 1) * cfg.n], clean["x"][p * cfg.n:(p + 1) * cfg.n])
    dev = {key: torch.from_numpy(np.ascontiguousarray(v)).cuda() for key, v in d.items() if key in "cAbGh"}
    hdd = S.SqrHandle(cfg.cones, cfg.n, cfg.m, cfg.k, dev["A"], dev["G"],
                      torch.zeros(B, dtype=torch.uint8, device="cuda"))
    gd = hdd.solve_socp(dev["c"], dev["b"], dev["h"])
    torch.cuda.synchronize()
    for key in ("x", "y", "z", "s", "iters", "status", "res"):
        assert np.array_equal(gd[key].cpu().numpy(), clean[key]), key


def test_scaling_at_a_boundary_iterate(kats, oracle):
    """A POC element on the cone boundary (s_i z_i = 0): the square roots of
    the scaling come from one Newton-refined 1/sqrt(s z), which is inf there;
    the reference's IEEE sqrt gives lambda_i = sqrt(s z) = 0 and
    wbs_i = sqrt(s/z) = 0 (s_i = 0) or inf (z_i = 0), and so must the device
    (not 0 * inf = NaN).  The other entries stay within 1e-12 of the oracle.
    Both plugins then report the factorisation failure where the reference's
    cholesky! throws (W^-2 has an infinite entry): status 2."""
    q = kats["sqr_scaling"]
    cones = [tuple(c) for c in q["cones"]]
    assert cones[0][0] == 0  # a POC block first
    G = np.array(q["G"], dtype=np.float64)
    k, n = G.shape
    s0, z0 = np.array(q["pairs"][0]["s"], float), np.array(q["pairs"][0]["z"], float)
    s1, z1 = s0.copy(), z0.copy()
    s1[0] = 0.0  # lambda_0 = 0, wbs_0 = 0
    s2, z2 = s0.copy(), z0.copy()
    z2[0] = 0.0  # lambda_0 = 0, wbs_0 = inf
    S_, Z_ = [s1, s2], [z1, z2]
    B = 2
    h = S.SqrHandle(cones, n, 0, k, None, np.tile(G.ravel(order="F"), B))
    st = h.setup_iter(np.concatenate(S_), np.concatenate(Z_))
    sc = h.scaling()
    for p in range(B):
        ref = oracle.compute_scaling(cones, S_[p], Z_[p])
        for key in ("l", "wbs"):
            got, want = np.asarray(sc[key][p]), np.asarray(ref[key])
            assert got[0] == want[0], (p, key, got, want)  # the boundary element: 0 or inf exactly
            assert np.abs(got[1:] - want[1:]).max() < 1e-12, (p, key, got, want)
    # the factorisation outcome as the oracle's (s_0 = 0: W^-2 has an infinite
    # entry, cholesky! throws; z_0 = 0: that row drops out of H), for both plugins
    zr = lambda q: np.zeros(q)  # noqa: E731
    A0 = np.zeros((0, n))
    want_sqr = [oracle.sqr_kkt_single(cones, A0, G, False, S_[p], Z_[p], zr(n), zr(0), zr(k), zr(k))["status"]
                for p in range(B)]
    want_dense = [oracle.kkt_single(cones, A0, G, False, S_[p], Z_[p], zr(n), zr(0), zr(k), zr(k))["status"]
                  for p in range(B)]
    assert want_sqr[0] == 2 and want_dense[0] == 2, (want_sqr, want_dense)
    assert st.tolist() == want_sqr, (st, want_sqr)
    d = S.DenseHandle(cones, n, 0, k, None, np.tile(G.ravel(order="F"), B))
    assert d.setup_iter(np.concatenate(S_), np.concatenate(Z_)).tolist() == want_dense
    d.close()
