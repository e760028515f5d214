"""Problem builders shared by the tests (reference test problems, synthetic configs)."""
import numpy as np


def kat_problem(q):
    """(cones, c, A, b, G, h) from a reference_kats.json entry (runtests.jl problems)."""
    c = np.array(q["c"], dtype=np.float64)
    n = len(c)
    A = np.array(q["A"], dtype=np.float64).reshape(-1, n)
    b = np.array(q["b"], dtype=np.float64)
    G = np.array(q["G"], dtype=np.float64)
    h = np.array(q["h"], dtype=np.float64)
    cones = [tuple(x) for x in q["cones"]]
    return cones, c, A, b, G, h


def optimal_control(N=50):
    """'Linear optimal control' of runtests.jl:204-244 (n=3N, m=2N+2, k=N, one SOC(0,N))."""
    n = 3 * N
    c = np.zeros(n)
    c[-1] = 1.0
    vel = np.arange(0, N)
    pos = np.arange(N, 2 * N)
    force = np.arange(2 * N, 3 * N - 1)
    A = np.zeros((2 * N + 2, n))
    b = np.zeros(2 * N + 2)
    A[vel[0], vel[0]] = 1.0
    b[vel[0]] = 1.0
    A[pos[0], pos[0]] = 1.0
    for stp in range(1, N):
        A[vel[stp], vel[stp]] = -1.0
        A[vel[stp], vel[stp - 1]] = 1.0
        A[vel[stp], force[stp - 1]] = 1.0
        A[pos[stp], pos[stp]] = -1.0
        A[pos[stp], pos[stp - 1]] = 1.0
        A[pos[stp], vel[stp - 1]] = 1.0
    A[2 * N, vel[N - 1]] = 1.0
    A[2 * N + 1, pos[N - 1]] = 1.0
    G = np.zeros((N, n))
    G[0, n - 1] = -1.0
    for i in range(N - 1):
        G[i + 1, 2 * N + i] = -1.0
    h = np.zeros(N)
    return [(1, 0, N)], c, A, b, G, h


def batch_problem(flat, B, n, m, k, p):
    """Problem p of a flat batch (include/socp.h layout) as dense row-major matrices."""
    A = flat["A"].reshape(B, m * n)[p].reshape(n, m).T if m else np.zeros((0, n))
    G = flat["G"].reshape(B, k * n)[p].reshape(n, k).T
    return (flat["c"].reshape(B, n)[p], A, flat["b"].reshape(B, m)[p] if m else np.zeros(0), G,
            flat["h"].reshape(B, k)[p])


def random_cones(rng, k, allow_poc=True):
    """Random contiguous POC-then-SOC cone list summing to k."""
    cones = []
    off = 0
    if allow_poc and rng.random() < 0.6:
        d = int(rng.integers(1, max(2, k // 2)))
        cones.append((0, 0, d))
        off = d
    while off < k:
        d = int(min(k - off, rng.integers(2, 33)))
        if d == 1 and cones and cones[-1][0] == 1:
            cones[-1] = (1, cones[-1][1], cones[-1][2] + 1)
            off += 1
            continue
        cones.append((1, off, d))
        off += d
    return cones


def perturb_G(G, seed):
    """Every entry of G one ulp up or down (seeded coin): a change of the data at
    the size of one rounding (tests/golden/make_chaos_floor.py uses the same)."""
    G = np.asarray(G, dtype=np.float64)
    up = np.random.default_rng(seed).integers(0, 2, G.size).astype(bool).reshape(G.shape)
    return np.where(up, np.nextafter(G, np.inf), np.nextafter(G, -np.inf))


def order_floor_traces(oracle, cones, c, A, b, G, h, K, flags, seeds=(1, 2, 3)):
    """The oracle's iterates 1..K in one operation order (flags) and, per
    iterate and vector, the largest relative change under a one-ulp
    perturbation of G over `seeds`: the rounding floor of a comparison with
    another implementation of the same order.  Returns (iterates[t] = (x, z, s),
    floor[t] = {"x", "z", "s"})."""
    P = oracle.Params(maxit=K, tol=0.0, flags=flags)

    def states(Gx):
        r = oracle.solve_trace(cones, c, A, b, Gx, h, sing=False, params=P, max_trace=K + 1)
        st = list(r["trace"][:r["iters"]]) + [(r["x"], r["y"], r["z"], r["s"])]
        return [(x, z, s) for x, y, z, s in st]

    base = states(G)
    floor = [{"x": 0.0, "z": 0.0, "s": 0.0} for _ in base]
    for sd in seeds:
        pert = states(perturb_G(G, sd))
        for t, (u, v) in enumerate(zip(base, pert)):
            for i, key in enumerate("xzs"):
                e = np.linalg.norm(u[i] - v[i]) / np.linalg.norm(u[i])
                floor[t][key] = max(floor[t][key], float(e))
    return base, floor


# A kernel-order iterate may differ from the oracle's in the same order by the
# rounding of a different summation order; its floor is the oracle's own
# sensitivity to one rounding (every G entry +-1 ulp, three seeds).  The gate is
# FLOOR_FACTOR times that floor (an order of magnitude: one ulp of the data is
# one rounding, the kernel's order differs from the oracle's in many), plus
# FLOOR_ABS for the first iterates, whose floor is a few ulps.
FLOOR_FACTOR, FLOOR_ABS = 10.0, 1e-13


def trajectory_at_floor(oracle, cfg, d, B, K, flags, solve):
    """Iterates 1..K of `solve(maxit)` (a batch of B problems of config cfg,
    generator data d) against the oracle in operation order `flags`, each
    vector gated by FLOOR_FACTOR * its one-rounding floor + FLOOR_ABS.
    Returns the (ratio, K, problem, vector, error, floor) rows, worst first."""
    ref = []
    for p in range(B):
        A = d["A"][p * cfg.m * cfg.n:(p + 1) * cfg.m * cfg.n].reshape(cfg.n, cfg.m).T
        G = d["G"][p * cfg.k * cfg.n:(p + 1) * cfg.k * cfg.n].reshape(cfg.n, cfg.k).T
        ref.append(order_floor_traces(oracle, cfg.cones, d["c"][p * cfg.n:(p + 1) * cfg.n], A,
                                      d["b"][p * cfg.m:(p + 1) * cfg.m], G, d["h"][p * cfg.k:(p + 1) * cfg.k],
                                      K, flags))
    rows = []
    for k_ in range(1, K + 1):
        g = solve(k_)
        assert (g["status"] == 1).all(), (k_, g["status"])  # every problem at maxit: no early stop
        for p in range(B):
            it, fl = ref[p][0][k_], ref[p][1][k_]
            for i, (key, L) in enumerate((("x", cfg.n), ("z", cfg.k), ("s", cfg.k))):
                a_, b_ = np.asarray(g[key][p * L:(p + 1) * L]), it[i]
                e = float(np.linalg.norm(a_ - b_) / np.linalg.norm(b_))
                rows.append((e / (FLOOR_FACTOR * fl[key] + FLOOR_ABS), k_, p, key, e, fl[key]))
    return sorted(rows, reverse=True)
