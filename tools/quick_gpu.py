import sys, os, json, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "socp.jl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import socp_amd as S
import oracle as O
from socp_amd.configs import C0B, C1, C2

K = json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "reference_kats.json")))
g = K["kkt_golden"]
G = np.array(g["G"])
out = S.batch_kkt_solve(g["cones"], 3, 0, 4, None, G.ravel(order="F"), None, np.array(g["s"]), np.array(g["z"]),
                        np.array(g["dx"]), None, np.array(g["dz"]), np.array(g["ds"]))
print("KKT golden status", out["status"], {kk: float(np.abs(out[kk] - np.array(g[kk])).max()) for kk in ("cx", "cz", "cs")})
for name in ("soc1", "soc2", "soc3"):
    q = K[name]
    prob = S.Problem(q["c"], q["A"], q["b"], q["G"], q["h"], [tuple(c) for c in q["cones"]])
    ss = S.SolverState(prob, S.DenseSolver(prob))
    try:
        st = S.solve_socp(prob, ss)
        print(name, ss.status, ss.iters, st.x, np.linalg.norm(st.x - np.array(q["x_expect"])))
    except Exception as e:
        print(name, "raised", repr(e), ss.status, ss.iters)
for cfg, B in ((C0B, 64), (C1, 256), (C2, 256)):
    d = O.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    t0 = time.time()
    r = O.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"], sing=None)
    t1 = time.time()
    gpu = S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"], None, res=True)
    t2 = time.time()
    agree = (gpu["status"] == r["status"])
    conv = (r["status"] == 0) & (gpu["status"] == 0)
    dx = np.abs(gpu["x"].reshape(B, -1) - r["x"].reshape(B, -1)).max(axis=1)
    print(cfg.name, "oracle status", np.bincount(r["status"], minlength=5), "gpu status", np.bincount(gpu["status"], minlength=5),
          "agree", agree.mean(), "iters diff max", np.abs(gpu["iters"] - r["iters"])[conv].max() if conv.any() else None,
          "x diff (both conv) max", dx[conv].max() if conv.any() else None, "cpu %.3fs gpu %.3fs" % (t1 - t0, t2 - t1))
    # fixed-K
    rk = O.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"], params=O.Params(maxit=3, tol=0.0))
    gk = S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"], None, maxit=3, tol=0.0)
    rel = np.linalg.norm(gk["x"].reshape(B, -1) - rk["x"].reshape(B, -1), axis=1) / np.linalg.norm(rk["x"].reshape(B, -1), axis=1)
    print("   fixed-K=3 status", np.bincount(gk["status"], minlength=5), "rel x diff max", rel.max())
