"""Multi-tile KKT diagnostic: dumps H and -H^-1 from the device (KKT mode debug
hook) for C1/C2-shaped problems and reports the error per 16x16 tile against
numpy, plus the KKT solution against the oracle."""
import sys, os
os.environ["SOCP_AMD_LIB"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "socp.jl_amd", "lib", "libsocp_diag.so")
import numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "socp.jl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import socp_amd as S
from socp_amd import _lib
import oracle as O
from socp_amd.configs import C1, C2

np.set_printoptions(precision=2, linewidth=160)
S.default_context()
for cfg in (C1, C2):
    B = 2
    d = O.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    n, m, k = cfg.n, cfg.m, cfg.k
    cones = list(cfg.cones)
    A = d["A"].reshape(B, m * n)[0].reshape(n, m).T
    G = d["G"].reshape(B, k * n)[0].reshape(n, k).T
    buf = torch.zeros(2 * n * n + 2 * k + n * m + m * m, dtype=torch.float64, device="cuda")
    _lib.load().socp_debug_set_kkt_dump(_lib.ptr(buf))
    e = O.make_e(cones, k)
    rng = np.random.default_rng(0)
    for label, (s, z) in (("identity", (e.copy(), e.copy())),
                          ("generic", (e + 0.1 * rng.random(k), e + 0.1 * rng.random(k)))):
        rhs = (rng.standard_normal(n), rng.standard_normal(m), rng.standard_normal(k), rng.standard_normal(k))
        gg = S.batch_kkt_solve(cones, n, m, k, A.ravel(order="F"), G.ravel(order="F"), np.zeros(1, np.uint8),
                               s, z, *rhs)
        torch.cuda.synchronize()
        D = buf.cpu().numpy()
        Hg = D[:n * n].reshape(n, n)
        Lig = D[n * n:2 * n * n].reshape(n, n)
        o0 = 2 * n * n + 2 * k
        ALg = D[o0:o0 + n * m].reshape(n, m)
        Sg = D[o0 + n * m:o0 + n * m + m * m].reshape(m, m)
        o = O.kkt_single(cones, A, G, False, s, z, *rhs, want_H=True)
        Ho = o["H"]
        Hinv = np.linalg.inv(Ho)
        print(f"== {cfg.name} {label}: status {gg['status']}")
        nt = (n + 15) // 16
        eh = np.zeros((nt, nt)); el = np.zeros((nt, nt))
        for i in range(nt):
            for j in range(nt):
                sl = (slice(16 * i, 16 * i + 16), slice(16 * j, 16 * j + 16))
                eh[i, j] = np.abs(Hg[sl] - Ho[sl]).max() / np.abs(Ho).max()
                el[i, j] = np.abs(Lig[sl] - Hinv[sl]).max() / np.abs(Hinv).max()
        print("  H tile err\n", eh)
        print("  Li tile err (vs +inv)\n", el)
        print("  Li tile err (vs -inv)\n", np.array([[np.abs(Lig[16*i:16*i+16, 16*j:16*j+16] + Hinv[16*i:16*i+16, 16*j:16*j+16]).max() / np.abs(Hinv).max() for j in range(nt)] for i in range(nt)]))
        ALr = Hinv @ A.T
        Sr = A @ ALr
        print("  ALi' rel err per 16-row block", [float(np.abs(ALg[16*i:16*i+16] - ALr[16*i:16*i+16]).max() / np.abs(ALr).max()) for i in range(nt)])
        print("  ALi' rel err vs -Hinv A'", float(np.abs(ALg + ALr).max() / np.abs(ALr).max()))
        print("  S rel err (lower)", float(np.abs(np.tril(Sg) - np.tril(Sr)).max() / np.abs(Sr).max()), "eig S_gpu", np.linalg.eigvalsh(np.tril(Sg) + np.tril(Sg, -1).T)[:3])
        for key in ("cx", "cy", "cz", "cs"):
            if key in gg and key in o and len(o[key]):
                print(f"  {key} rel err {np.linalg.norm(gg[key] - o[key]) / max(np.linalg.norm(o[key]), 1e-300):.2e}")
