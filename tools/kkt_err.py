import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "socp.jl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import socp_amd as S
import oracle as O
from socp_amd.configs import C1, C2

def kkt_res(cones, A, G, s, z, sol, rhs):
    sc = O.compute_scaling(cones, s, z)
    W, l = sc["W"], sc["l"]
    cx, cy, cz, cs = sol
    dx, dy, dz, ds = rhs
    r1 = A.T @ cy + G.T @ cz - dx
    r2 = A @ cx - dy
    r3 = G @ cx + cs - dz
    r4 = O.vprod(cones, l, W @ cz + np.linalg.solve(W.T, cs)) - ds
    return [np.linalg.norm(r) / max(np.linalg.norm(q), 1e-300) for r, q in ((r1, dx), (r2, dy if len(dy) else np.ones(1)), (r3, dz), (r4, ds))]

for cfg in (C1, C2):
    B = 4
    d = O.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    n, m, k = cfg.n, cfg.m, cfg.k
    for p in range(2):
        A = d["A"].reshape(B, m * n)[p].reshape(n, m).T; G = d["G"].reshape(B, k * n)[p].reshape(n, k).T
        tr = O.solve_trace(cfg.cones, d["c"].reshape(B, n)[p], A, d["b"].reshape(B, m)[p], G, d["h"].reshape(B, k)[p], params=O.Params(maxit=12, tol=0.0), max_trace=13)
        rng = np.random.default_rng(p)
        for t in range(2, min(len(tr["trace"]), 12)):
            x, y, z, s = tr["trace"][t]
            rhs = (rng.standard_normal(n), rng.standard_normal(m), rng.standard_normal(k), rng.standard_normal(k))
            o = O.kkt_single(cfg.cones, A, G, False, s, z, *rhs, want_H=True)
            gg = S.batch_kkt_solve(cfg.cones, n, m, k, A.ravel(order="F"), G.ravel(order="F"), np.zeros(1, np.uint8), s, z, *rhs)
            kap = np.linalg.cond(o["H"])
            eo = kkt_res(cfg.cones, A, G, s, z, (o["cx"], o["cy"], o["cz"], o["cs"]), rhs)
            eg = kkt_res(cfg.cones, A, G, s, z, (gg["cx"], gg["cy"], gg["cz"], gg["cs"]), rhs)
            print(f"{cfg.name} p{p} it{t} kappa(H)={kap:.1e} oracle relres " + " ".join(f"{v:.1e}" for v in eo) + " | gpu " + " ".join(f"{v:.1e}" for v in eg))
