"""Generates tests/golden/c2_refrule_outcomes.json: the oracle's outcome of the
first 4,096 C2 problems under the reference's stopping rule (solver.jl:105,122:
maxit = 40, absolute tol = 1e-5), per problem: status, iterations, final
||rd||, ||rp||, z's -- once in the reference's operation order and once in the
structured order the HIP kernels use (oracle flag F_STRUCTURED), with the
explicit inverse and -- as the register kernel runs C2 (m <= 16) -- with
triangular solves (F_STRUCTURED | F_CHOLSOLVE).  The GPU test
tests/test_gpu_outcomes.py compares the HIP histogram and per-problem outcomes
with these (allowed gaps: DESIGN.md §9).

usage: python tests/golden/make_outcomes.py   (about a minute on 8 cores)
"""
import base64
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


def b64(a, dt):
    return base64.b64encode(np.ascontiguousarray(a, dtype=dt).tobytes()).decode()


def main():
    O.build()
    cfg = C2
    d = O.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    out = {"_doc": __doc__.strip().splitlines()[0], "config": cfg.name, "seed": cfg.seed, "batch": B,
           "maxit": 40, "tol": 1e-5, "runs": {}}
    sing = np.zeros(B, np.uint8)  # the generator's G (k > n, uniform entries) has full column rank
    for name, flags in (("reference_order", 0), ("structured", O.F_STRUCTURED),
                        ("structured_chol", O.F_STRUCTURED | O.F_CHOLSOLVE)):
        r = O.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"], sing=sing,
                          params=O.Params(maxit=40, tol=1e-5, flags=flags), nthreads=os.cpu_count())
        out["runs"][name] = {"status": b64(r["status"], "<i1"), "iters": b64(r["iters"], "<i1"),
                             "res": b64(r["res"], "<f8"),
                             "histogram": np.bincount(r["status"], minlength=5).tolist()}
        print(name, out["runs"][name]["histogram"], "mean iters", float(r["iters"].mean()))
    path = os.path.join(HERE, "c2_refrule_outcomes.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print(f"wrote {path}: {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
