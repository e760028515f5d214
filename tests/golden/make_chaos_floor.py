"""Generates tests/golden/c2_chaos_floor.json: the chaos floor of the outcome
comparisons in tests/test_gpu_outcomes.py and test_gpu_parity.py::test_outcome_parity
 -- how far the oracle's outcomes move under a rounding-only
perturbation, measured on the same first 4,096 C2 problems under the reference's
stopping rule (solver.jl:105,122: maxit = 40, absolute tol = 1e-5).

The perturbation: every entry of G moved by one ulp (np.nextafter), up or down
by a seeded coin, for three seeds -- a change of the data at the level of one
rounding, i.e. the same size as the difference between two summation orders.
For each operation order of the oracle (reference_order: flags 0;
structured: F_STRUCTURED, Li = H^-1 formed; structured_chol: F_STRUCTURED |
F_CHOLSOLVE, the register kernel's order) the unperturbed run is compared with
each perturbed run ("self" floor), and for the cross-order gate (HIP in the
Cholesky order against the reference-order oracle) the structured_chol runs,
unperturbed and perturbed, are compared with the unperturbed reference-order
run ("cross" floor) -- on all 4,096 and on the first 256 (the P5 test's batch).

Statistics (a, b = two runs):
  same      fraction of problems with the same status
  of_conv   of the problems b converges on, the fraction a converges on
            (self: the smaller of the two directions)
  maxit     of the problems b converges on, the fraction a stops at maxit
  iters1    where both converge, the fraction with |iters_a - iters_b| <= 1
  dconv     |converged_a - converged_b| / B;  dfail likewise for the failures
            (chol(H) + chol(S) + domain)
The floor of a statistic is its worst value over the perturbed comparisons
(min for fractions that should be high, max for dconv / dfail / maxit).  The
gates are that floor with one point of slack (GATE_SLACK = 0.01).

usage: python tests/golden/make_chaos_floor.py   (about two minutes on 8 cores)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "socp.jl_amd"))

import oracle as O  # noqa: E402
from socp_amd.configs import C2  # noqa: E402

B = 4096
SEEDS = (1, 2, 3)
GATE_SLACK = 0.01
ORDERS = (("reference_order", 0), ("structured", O.F_STRUCTURED),
          ("structured_chol", O.F_STRUCTURED | O.F_CHOLSOLVE))


def perturb_G(G, seed):
    """Every entry one ulp up or down (seeded coin)."""
    up = np.random.default_rng(seed).integers(0, 2, G.size).astype(bool)
    return np.where(up, np.nextafter(G, np.inf), np.nextafter(G, -np.inf))


def stats(a, b, symmetric):
    """Outcome agreement of run a against run b (dicts of status, iters)."""
    sa, sb = a["status"], b["status"]
    ca, cb = sa == 0, sb == 0
    of_conv = float((ca[cb]).mean()) if cb.any() else 1.0
    if symmetric and ca.any():
        of_conv = min(of_conv, float((cb[ca]).mean()))
    both = ca & cb
    di = np.abs(a["iters"][both] - b["iters"][both])
    fail = lambda s: int(((s >= 2) & (s <= 4)).sum())  # noqa: E731
    n = len(sa)
    return {"same": float((sa == sb).mean()), "of_conv": of_conv,
            "maxit": float((sa[cb] == 1).mean()) if cb.any() else 0.0,
            "iters1": float((di <= 1).mean()) if di.size else 1.0,
            "dconv": abs(int(ca.sum()) - int(cb.sum())) / n, "dfail": abs(fail(sa) - fail(sb)) / n}


def floor(rows):
    lo = ("same", "of_conv", "iters1")
    return {key: (min(r[key] for r in rows) if key in lo else max(r[key] for r in rows)) for key in rows[0]}


def solve_all(nthreads=None):
    cfg = C2
    d = O.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    sing = np.zeros(B, np.uint8)
    runs = {}
    for name, flags in ORDERS:
        P = O.Params(maxit=40, tol=1e-5, flags=flags)
        for seed in (0,) + SEEDS:
            G = d["G"] if seed == 0 else perturb_G(d["G"], seed)
            r = O.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], G, d["h"], sing=sing,
                              params=P, nthreads=nthreads or os.cpu_count())
            runs[(name, seed)] = {"status": r["status"], "iters": r["iters"]}
            print(name, seed, np.bincount(r["status"], minlength=5).tolist(), flush=True)
    return runs


def main():
    O.build()
    runs = solve_all()
    out = {"_doc": __doc__.strip().splitlines()[0], "config": "C2", "seed": C2.seed, "batch": B, "maxit": 40,
           "tol": 1e-5, "perturbation": "G entries +-1 ulp (np.nextafter), seeded coin", "seeds": list(SEEDS),
           "gate_slack": GATE_SLACK, "histograms": {}, "self": {}, "cross": {}}
    for (name, seed), r in runs.items():
        out["histograms"][f"{name}/{seed}"] = np.bincount(r["status"], minlength=5).tolist()
    for name, _ in ORDERS:
        rows = [stats(runs[(name, s)], runs[(name, 0)], symmetric=True) for s in SEEDS]
        out["self"][name] = {"floor": floor(rows), "per_seed": rows}
    for sub, nb in (("all", B), ("first256", 256)):
        cut = lambda r: {key: v[:nb] for key, v in r.items()}  # noqa: E731
        rows = [stats(cut(runs[("structured_chol", s)]), cut(runs[("reference_order", 0)]), symmetric=False)
                for s in (0,) + SEEDS]
        out["cross"][f"structured_chol_vs_reference_order/{sub}"] = {"floor": floor(rows), "per_run": rows}
    path = os.path.join(HERE, "c2_chaos_floor.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({key: out[key] for key in ("self", "cross")}, indent=1))
    print(f"wrote {path}")


if __name__ == "__main__":
    main()
