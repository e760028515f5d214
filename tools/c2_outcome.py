"""C2 outcome diagnosis: where the oracle converges but the device does not,
report both iteration counts, the device residual history and kappa(H) along
the oracle trajectory."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "socp.jl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import socp_amd as S
import oracle as O
from problems import batch_problem
from socp_amd.configs import C2

cfg, B = C2, 256
n, m, k = cfg.n, cfg.m, cfg.k
d = O.generate(cfg.cones, B, n, m, k, cfg.seed)
r = O.batch_solve(cfg.cones, n, m, k, d["c"], d["A"], d["b"], d["G"], d["h"])
g = S.batch_solve(cfg.cones, n, m, k, d["c"], d["A"], d["b"], d["G"], d["h"], None, res=True)
print("oracle status", np.bincount(r["status"], minlength=5), "gpu", np.bincount(g["status"], minlength=5))
tab = np.zeros((5, 5), int)
for a, b in zip(r["status"], g["status"]):
    tab[a, b] += 1
print("rows oracle status, cols gpu status\n", tab)
bad = np.where((r["status"] == 0) & (g["status"] != 0))[0]
print("oracle-converged, gpu not:", bad.size)
for p in bad[:8]:
    # per-iteration device residual: rerun with maxit=K
    hist = []
    for K in range(max(0, g["iters"][p] - 4), g["iters"][p] + 1):
        c, A, b, G, h = batch_problem(d, B, n, m, k, p)
        o = S.batch_solve(cfg.cones, n, m, k, c, A.ravel(order="F"), b, G.ravel(order="F"), h, None,
                          maxit=K, tol=0.0, res=True)
        hist.append((K, int(o["status"][0]), float(o["res"].sum())))
    c, A, b, G, h = batch_problem(d, B, n, m, k, p)
    tr = O.solve_trace(cfg.cones, c, A, b, G, h, max_trace=41)
    print(f"p={p} oracle iters {r['iters'][p]} res {r['res'].reshape(B, 3)[p].sum():.2e} | gpu status {g['status'][p]} "
          f"iters {g['iters'][p]} res {g['res'].reshape(B, 3)[p].sum():.2e}; gpu hist {hist}")
    rr = [np.linalg.norm(A.T @ y + G.T @ z + c) + np.linalg.norm(A @ x - b) + z @ s for x, y, z, s in tr["trace"]]
    print("    oracle res history", " ".join(f"{x:.1e}" for x in rr))
ok = r["status"] == 0
both = ok & (g["status"] == 0)
print("iters diff on both-converged:", np.bincount(np.abs(g["iters"] - r["iters"])[both]))
