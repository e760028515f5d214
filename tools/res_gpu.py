import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "socp.jl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import socp_amd as S
import oracle as O
from socp_amd.configs import C1
cfg, B = C1, 8
d = O.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
for K in (1, 2, 3, 4, 5, 6, 7):
    r = O.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"], params=O.Params(maxit=K, tol=0.0))
    g = S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"], None, maxit=K, tol=0.0, res=True)
    print(K, "oracle res", r["res"][:3].tolist())
    print(K, "gpu    res", g["res"].reshape(B, 3)[:3].tolist())
g = S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"], None, res=True)
print("tol mode gpu", g["status"], g["iters"], g["res"].reshape(B, 3)[:3].tolist())
r = O.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"])
print("tol mode oracle", r["status"], r["iters"], r["res"][:3].tolist())
