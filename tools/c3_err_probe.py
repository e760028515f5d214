"""Exploration (not a test): C3 last-shard errors of the HIP solve vs the
reference-order and the Cholesky-order (F_STRUCTURED | F_CHOLSOLVE) oracle,
with the worst kappa_2(H) on each oracle trajectory."""
import sys
import numpy as np
import torch
sys.path[:0] = ["tests", "socp.jl_amd", "."]
import socp_amd as S  # noqa: E402
from oracle import oracle as O  # noqa: E402
from socp_amd.configs import C3 as cfg  # noqa: E402
from problems import batch_problem  # noqa: E402

B, K = 65536, 8
first = 7 * B
c, A, b, G, h = S.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed, first_problem=first)
out = S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, c, A, b, G, h, torch.zeros(B, dtype=torch.uint8, device=G.device),
                    maxit=K, tol=0.0)
flat = {k_: t.cpu().numpy() for k_, t in zip("c A b G h".split(), (c, A, b, G, h))}
rel = lambda a, b_: np.linalg.norm(a - b_) / np.linalg.norm(b_)  # noqa: E731
for p in np.random.default_rng(7).choice(B, 24, replace=False):
    pc, pA, pb, pG, ph = batch_problem(flat, B, cfg.n, cfg.m, cfg.k, p)
    row = []
    for fl in (0, O.F_STRUCTURED | O.F_CHOLSOLVE):
        r = O.solve_trace(cfg.cones, pc, pA, pb, pG, ph, sing=False, params=O.Params(maxit=K, tol=0.0, flags=fl))
        kap = max(np.linalg.cond(O.kkt_single(cfg.cones, pA, pG, False, s, z, np.zeros(cfg.n), np.zeros(cfg.m),
                                              np.zeros(cfg.k), np.zeros(cfg.k), want_H=True)["H"])
                  for _, _, z, s in r["trace"][:K])
        e = [rel(out[k_][p * d:(p + 1) * d].cpu().numpy(), r[k_]) for k_, d in (("x", cfg.n), ("z", cfg.k), ("s", cfg.k))]
        row.append("kap %.1e x %.1e z %.1e s %.1e" % (kap, *e))
    print(p, " | ".join(row), flush=True)
