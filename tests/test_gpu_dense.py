"""The split plugin boundary (socp_dense_*): DenseSolver construction, then
setup_iter once and solve_kkt as often as the solver needs (densesolver.jl:
19-38, 41-52, 54-90; solver.jl calls solve_kkt twice per iteration).

Gates:
  * two solve_kkt calls after one setup_iter equal the fused entry
    (socp_batch_kkt_solve) bitwise, for the register kernel (C2 shape, one
    record per problem) and the blocked kernel (forced, and at the C4 shape);
  * per-call host-to-device traffic is O(n + m + k) per problem: exactly
    2k doubles for setup_iter and n + m + 2k for solve_kkt;
  * device-tensor handles give the host results bitwise;
  * a problem whose setup fails reports the setup status and NaN solutions
    without disturbing its neighbours; solve_kkt before setup_iter is refused;
  * the reference's KKT golden (runtests.jl:95-128) through the mirror surface
    with the split calls.
"""
import numpy as np
import pytest

import socp_amd as S
from socp_amd.configs import C2, C4

pytestmark = pytest.mark.gpu


def iterates(cfg, B, maxit, seed=None, force_large=False):
    """Interior (s, z) after `maxit` solver iterations of B generated problems."""
    d = S.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed if seed is None else seed)
    c, A, b, G, h = (t.cpu().numpy() for t in d)
    out = S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, c, A, b, G, h, np.zeros(B, np.uint8), maxit=maxit,
                        tol=0.0, force_large=force_large)
    return dict(A=A, G=G, s=out["s"], z=out["z"])


def rhs(cfg, B, seed):
    rng = np.random.default_rng(seed)
    return [rng.standard_normal(B * q) for q in (cfg.n, cfg.m, cfg.k, cfg.k)]


def fused(cfg, it, r, force_large=False):
    B = len(it["s"]) // cfg.k
    return S.batch_kkt_solve(cfg.cones, cfg.n, cfg.m, cfg.k, it["A"], it["G"], np.zeros(B, np.uint8), it["s"],
                             it["z"], *r, force_large=force_large)


def check_split_equals_fused(cfg, B, maxit, force_large=False):
    it = iterates(cfg, B, maxit, force_large=force_large)
    h = S.DenseHandle(cfg.cones, cfg.n, cfg.m, cfg.k, it["A"], it["G"], np.zeros(B, np.uint8),
                      force_large=force_large)
    st = h.setup_iter(it["s"], it["z"])
    assert (st == 0).all()
    assert h.h2d_bytes == B * 2 * cfg.k * 8
    for seed in (1, 2):  # the affine and the combined solve of one iteration
        r = rhs(cfg, B, seed)
        got = h.solve_kkt(*r)
        assert h.h2d_bytes == B * (cfg.n + cfg.m + 2 * cfg.k) * 8
        ref = fused(cfg, it, r, force_large=force_large)
        assert np.array_equal(got["status"], ref["status"])
        for key in ("cx", "cy", "cz", "cs"):
            assert np.array_equal(got[key], ref[key]), (key, seed)
    return h, it


def test_split_equals_fused_c2_register_kernel():
    h, _ = check_split_equals_fused(C2, 512, 4)
    assert h.record_bytes < 64 * 1024  # H^-1 and S^-1 tiles + cone state (about 28 KB at C2)


def test_split_equals_fused_blocked_kernel():
    check_split_equals_fused(C2, 64, 4, force_large=True)


def test_split_equals_fused_c4():
    check_split_equals_fused(C4, 16, 3)


def test_setup_once_solve_many_is_stable():
    """The record is read-only to solve_kkt: the same right-hand side solved
    again after other solves gives the same bits."""
    cfg, B = C2, 128
    it = iterates(cfg, B, 3)
    h = S.DenseHandle(cfg.cones, cfg.n, cfg.m, cfg.k, it["A"], it["G"], np.zeros(B, np.uint8))
    h.setup_iter(it["s"], it["z"])
    r1 = rhs(cfg, B, 11)
    a = h.solve_kkt(*r1)
    for seed in (12, 13, 14):
        h.solve_kkt(*rhs(cfg, B, seed))
    b = h.solve_kkt(*r1)
    for key in ("cx", "cy", "cz", "cs"):
        assert np.array_equal(a[key], b[key])
    # a second setup at other iterates replaces the record
    it2 = iterates(cfg, B, 5)
    h.setup_iter(it2["s"], it2["z"])
    got = h.solve_kkt(*r1)
    ref = fused(cfg, dict(A=it["A"], G=it["G"], s=it2["s"], z=it2["z"]), r1)
    for key in ("cx", "cy", "cz", "cs"):
        assert np.array_equal(got[key], ref[key])


def test_device_handle_equals_host():
    import torch
    cfg, B = C2, 256
    it = iterates(cfg, B, 4)
    r = rhs(cfg, B, 5)
    hh = S.DenseHandle(cfg.cones, cfg.n, cfg.m, cfg.k, it["A"], it["G"], np.zeros(B, np.uint8))
    hh.setup_iter(it["s"], it["z"])
    ref = hh.solve_kkt(*r)
    T = lambda a, dt=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to("cuda", dt)  # noqa: E731
    hd = S.DenseHandle(cfg.cones, cfg.n, cfg.m, cfg.k, T(it["A"]), T(it["G"]), T(np.zeros(B, np.uint8), torch.uint8))
    st = hd.setup_iter(T(it["s"]), T(it["z"]))
    got = hd.solve_kkt(*(T(v) for v in r))
    torch.cuda.synchronize()
    assert hd.h2d_bytes == 0
    assert (st.cpu().numpy() == 0).all()
    for key in ("cx", "cy", "cz", "cs"):
        assert np.array_equal(got[key].cpu().numpy(), ref[key]), key
    with pytest.raises(TypeError):
        hd.solve_kkt(*r)


@pytest.mark.parametrize("force_large", [False, True])
def test_failed_setup_is_isolated(force_large):
    cfg, B = C2, 32
    it = iterates(cfg, B, 3, force_large=force_large)
    s = it["s"].copy()
    s[5 * cfg.k + 40] = 10.0 * s[5 * cfg.k + 32]  # problem 5: s leaves its second cone
    h = S.DenseHandle(cfg.cones, cfg.n, cfg.m, cfg.k, it["A"], it["G"], np.zeros(B, np.uint8),
                      force_large=force_large)
    st = h.setup_iter(s, it["z"])
    assert st[5] == S.DOMAIN_ERROR and (np.delete(st, 5) == 0).all()
    r = rhs(cfg, B, 3)
    got = h.solve_kkt(*r)
    assert got["status"][5] == S.DOMAIN_ERROR and (np.delete(got["status"], 5) == 0).all()
    assert np.isnan(got["cx"][5 * cfg.n:6 * cfg.n]).all()
    ref = fused(cfg, it, r, force_large=force_large)
    keep = np.ones(B, bool)
    keep[5] = False
    for key, q in (("cx", cfg.n), ("cy", cfg.m), ("cz", cfg.k), ("cs", cfg.k)):
        assert np.array_equal(got[key].reshape(B, q)[keep], ref[key].reshape(B, q)[keep]), key


def test_solve_before_setup_is_refused():
    cfg, B = C2, 4
    it = iterates(cfg, B, 1)
    h = S.DenseHandle(cfg.cones, cfg.n, cfg.m, cfg.k, it["A"], it["G"])
    with pytest.raises(S.SocpError, match="before setup_iter"):
        h.solve_kkt(*rhs(cfg, B, 0))


def test_mirror_split_calls_kkt_golden(kats):
    """runtests.jl:118-127 on the mirror: DenseSolver(prob), compute_scaling,
    setup_iter, then solve_kkt twice (the second with a scaled right-hand side,
    whose solution is the scaled first by linearity up to rounding)."""
    g = kats["kkt_golden"]
    cones = [S.POC(0, 1), S.SOC(1, 3)]
    prob = S.Problem(g["c"], np.zeros((0, 3)), [], g["G"], g["h"], cones)
    solver = S.DenseSolver(prob)
    scaling = S.compute_scaling(cones, S.Scaling(prob), g["s"], g["z"])
    st = S.State(prob, g["x"], [], g["z"], g["s"])
    S.setup_iter(solver, prob, st, scaling)
    dx, dz, ds = np.array(g["dx"]), np.array(g["dz"]), np.array(g["ds"])
    cx, cy, cz, cs = np.zeros(3), np.zeros(0), np.zeros(4), np.zeros(4)
    S.solve_kkt(solver, prob, st, scaling, dx, np.zeros(0), dz, ds, cx, cy, cz, cs)
    for key, v in (("cx", cx), ("cz", cz), ("cs", cs)):
        assert np.abs(v - np.array(g[key])).max() <= 1e-10, key
    cx2, cz2, cs2 = np.zeros(3), np.zeros(4), np.zeros(4)
    S.solve_kkt(solver, prob, st, scaling, 2 * dx, np.zeros(0), 2 * dz, 2 * ds, cx2, cy, cz2, cs2)
    assert np.abs(cx2 - 2 * cx).max() <= 1e-12 * max(1.0, np.abs(cx).max())
    assert solver.handle.h2d_bytes == (3 + 0 + 2 * 4) * 8
