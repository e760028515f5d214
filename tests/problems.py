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
