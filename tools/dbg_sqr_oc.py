"""Debug: the rank-update IPM on the runtests.jl optimal-control problem, K = 1..6 vs the oracle."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "socp.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import socp_amd as S
import oracle as O
from problems import optimal_control
cones, c, A, b, G, h = optimal_control(50)
n, m, k = len(c), A.shape[0], G.shape[0]
hd = S.SqrHandle(cones, n, m, k, A.ravel(order="F"), G.ravel(order="F"), np.ones(1, np.uint8))
for K in range(0, 7):
    g = hd.solve_socp(c, b, h, maxit=K, tol=0.0)
    r = O.solve_trace(cones, c, A, b, G, h, params=O.Params(maxit=K, tol=0.0, flags=O.F_SQR))
    ex = np.linalg.norm(g["x"] - r["x"]) / max(np.linalg.norm(r["x"]), 1e-300)
    ez = np.linalg.norm(g["z"] - r["z"]) / max(np.linalg.norm(r["z"]), 1e-300)
    print(K, "gpu", g["status"][0], g["iters"][0], g["res"], "oracle", r["status"], r["iters"], r["res"], "ex %.2e ez %.2e" % (ex, ez))
    if K >= 1:
        # the KKT solve at the oracle's iterate K-1 through the plugin
        tr = O.solve_trace(cones, c, A, b, G, h, params=O.Params(maxit=K - 1, tol=0.0, flags=O.F_SQR))
        st = hd.setup_iter(np.asarray(tr["s"]), np.asarray(tr["z"]))
        print("   setup at oracle iterate", K - 1, "status", st[0])
g = hd.solve_socp(c, b, h)
print("reference rule: gpu", g["status"][0], g["iters"][0], g["res"])
