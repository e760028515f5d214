import sys, os
os.environ["SOCP_AMD_LIB"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "socp.jl_amd", "lib", "libsocp_diag.so")
import numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "socp.jl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import socp_amd as S
from socp_amd import _lib
import oracle as O
from socp_amd.configs import C1
cfg = C1; B = 2
d = O.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
n, m, k = cfg.n, cfg.m, cfg.k; cones = list(cfg.cones)
A = d["A"].reshape(B, m*n)[0].reshape(n, m).T; G = d["G"].reshape(B, k*n)[0].reshape(n, k).T
tr = O.solve_trace(cones, d["c"].reshape(B, n)[0], A, d["b"].reshape(B, m)[0], G, d["h"].reshape(B, k)[0], params=O.Params(maxit=12, tol=0.0), max_trace=13)
buf = torch.zeros(2*n*n + 2*k + n*m + m*m, dtype=torch.float64, device="cuda")
S.default_context()
_lib.load().socp_debug_set_kkt_dump(_lib.ptr(buf))
rng = np.random.default_rng(0)
for t in range(2, 9):
    x, y, z, s = tr["trace"][t]
    rhs = (rng.standard_normal(n), rng.standard_normal(m), rng.standard_normal(k), rng.standard_normal(k))
    gg = S.batch_kkt_solve(cones, n, m, k, A.ravel(order="F"), G.ravel(order="F"), np.zeros(1, np.uint8), s, z, *rhs)
    D = buf.cpu().numpy()
    Hg = D[:n*n].reshape(n, n); Lig = D[n*n:2*n*n].reshape(n, n); lamg = D[2*n*n:2*n*n+k]; wbg = D[2*n*n+k:]
    o = O.kkt_single(cones, A, G, False, s, z, *rhs, want_H=True)
    sc = O.compute_scaling(cones, s, z)
    Ho = o["H"]
    print(f"it{t} kappa={np.linalg.cond(Ho):.1e} relH {np.linalg.norm(Hg-Ho)/np.linalg.norm(Ho):.1e} asym {np.linalg.norm(Hg-Hg.T)/np.linalg.norm(Hg):.1e} "
          f"|Hg Lig - I| {np.linalg.norm(Hg@Lig-np.eye(n)):.1e} |Ho inv(Ho)-I| {np.linalg.norm(Ho@np.linalg.inv(Ho)-np.eye(n)):.1e} "
          f"lam {np.linalg.norm(lamg-sc['l'])/np.linalg.norm(sc['l']):.1e} wb {np.linalg.norm(wbg-sc['wbs'])/np.linalg.norm(sc['wbs']):.1e}")
# save dumps for offline analysis
saves = {}
for t in range(2, 9):
    x, y, z, s = tr["trace"][t]
    rhs = (rng.standard_normal(n), rng.standard_normal(m), rng.standard_normal(k), rng.standard_normal(k))
    S.batch_kkt_solve(cones, n, m, k, A.ravel(order="F"), G.ravel(order="F"), np.zeros(1, np.uint8), s, z, *rhs)
    D = buf.cpu().numpy().copy()
    saves[f"H{t}"] = D[:n*n].reshape(n, n); saves[f"Li{t}"] = D[n*n:2*n*n].reshape(n, n)
np.savez(os.path.join(os.path.dirname(__file__), "..", "gpurun_out", "dbg_dump.npz"), **saves)
