import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "socp.jl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import socp_amd as S
import oracle as O
from socp_amd.configs import C0B, C1, C2

for cfg, B in ((C1, 32), (C2, 32)):
    d = O.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    print("==", cfg.name)
    for K in range(1, 14):
        r = O.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"], params=O.Params(maxit=K, tol=0.0))
        g = S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"], None, maxit=K, tol=0.0, res=True)
        def rel(a, b, w):
            a = a.reshape(B, -1); b = b.reshape(B, -1)
            return np.linalg.norm(a - b, axis=1) / np.maximum(np.linalg.norm(b, axis=1), 1e-300)
        rx, rz, rs = rel(g["x"], r["x"], cfg.n), rel(g["z"], r["z"], cfg.k), rel(g["s"], r["s"], cfg.k)
        ok = (r["status"] == 1) & (g["status"] == 1)
        print(f"K={K:2d} ostat={np.bincount(r['status'],minlength=5)} gstat={np.bincount(g['status'],minlength=5)} "
              f"relx med={np.median(rx[ok]) if ok.any() else -1:.2e} max={rx[ok].max() if ok.any() else -1:.2e} relz max={rz[ok].max() if ok.any() else -1:.2e} rels max={rs[ok].max() if ok.any() else -1:.2e} "
              f"gap o={np.median(r['res'][:,2]):.2e} g={np.median(g['res'].reshape(B,3)[:,2]):.2e}")
    # single problem detail at p=0
    p = 0
    n, m, k = cfg.n, cfg.m, cfg.k
    A = d["A"].reshape(B, m * n)[p].reshape(n, m).T; G = d["G"].reshape(B, k * n)[p].reshape(n, k).T
    tr = O.solve_trace(cfg.cones, d["c"].reshape(B, n)[p], A, d["b"].reshape(B, m)[p], G, d["h"].reshape(B, k)[p], params=O.Params(maxit=12, tol=0.0), max_trace=13)
    for t, (x, y, z, s) in enumerate(tr["trace"]):
        if t == 0: continue
        g = S.batch_solve(cfg.cones, n, m, k, d["c"].reshape(B, n)[p], d["A"].reshape(B, m * n)[p], d["b"].reshape(B, m)[p], d["G"].reshape(B, k * n)[p], d["h"].reshape(B, k)[p], None, maxit=1, tol=0.0,
                          warm=tr["trace"][t - 1])
        print(f"  teacher-forced step {t}: status {g['status'][0]} rel dx {np.linalg.norm(g['x'] - x) / np.linalg.norm(x):.2e} rel dz {np.linalg.norm(g['z'] - z) / np.linalg.norm(z):.2e} rel ds {np.linalg.norm(g['s'] - s) / np.linalg.norm(s):.2e}")
