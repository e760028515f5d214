"""Generates tests/golden/trajectories.json: oracle iterates the parity tests pin
(SURVEY.md §8(c) "Fixtures to commit").

Contents, per case: the problem (runtests.jl data from reference_kats.json, or a
(config, seed, problem index) of the device/oracle SplitMix64 generator, which
tests/test_gpu_parity.py::test_device_generator_bit_exact pins bit-exactly), the
oracle's (x, y, z, s) at the start of every iteration t (t = 0 is the initial
point of solver.jl:68-104) and kappa_2(H_t) of the dense KKT at that iterate.
Float arrays are base64 little-endian float64 (the file stays small and exact).

The oracle (oracle/socp_oracle.c) restates the reference's dense path; it is
pinned by every known-answer vector of test/runtests.jl (tests/test_oracle.py).

usage: python tests/golden/make_trajectories.py
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
sys.path.insert(0, os.path.dirname(HERE))

import oracle as O  # noqa: E402
from problems import kat_problem  # noqa: E402
from socp_amd.configs import C0B, C1, C2, C4  # noqa: E402


def b64(a):
    return base64.b64encode(np.ascontiguousarray(a, dtype="<f8").tobytes()).decode()


def kappa_H(cones, A, G, sing, s, z):
    n, m, k = G.shape[1], A.shape[0], G.shape[0]
    r = O.kkt_single(cones, A, G, sing, s, z, np.zeros(n), np.zeros(m), np.zeros(k), np.zeros(k), want_H=True)
    H = r["H"]
    if r["status"] != 0 or not np.isfinite(H).all():
        return None  # the factorisation failed at this iterate (status 2/3/4)
    return float(np.linalg.cond(H))


def case(name, cones, c, A, b, G, h, max_iters, source):
    n = len(c)
    A = np.asarray(A, dtype=np.float64).reshape(-1, n)
    G = np.asarray(G, dtype=np.float64)
    sing = O.sing_flag(G)
    r = O.solve_trace(cones, c, A, b, G, h, params=O.Params(maxit=max_iters, tol=0.0))
    # iterates past a numerical failure are not fixtures
    if r["status"] not in (0, 1):
        raise SystemExit(f"{name}: oracle status {r['status']} within {max_iters} iterations; lower max_iters")
    # trace[t], t < iters: the iterate at the start of iteration t; the state
    # after the last iteration is the returned (x, y, z, s)
    states = list(r["trace"][:r["iters"]]) + [(r["x"], r["y"], r["z"], r["s"])]
    its = []
    for x, y, z, s in states:
        its.append({"x": b64(x), "y": b64(y), "z": b64(z), "s": b64(s),
                    "kappa_H": kappa_H(cones, A, G, sing, s, z)})
    return {"name": name, "source": source, "cones": [list(map(int, t)) for t in cones], "n": n,
            "m": A.shape[0], "k": G.shape[0], "sing": bool(sing), "iterates": its}


def main():
    kats = json.load(open(os.path.join(HERE, "reference_kats.json")))
    out = {"_doc": __doc__.strip().splitlines()[0], "cases": []}
    for name in ("soc1", "soc2", "soc3"):
        cones, c, A, b, G, h = kat_problem(kats[name])
        out["cases"].append(case(name, cones, c, A, b, G, h, 12, {"kats": name}))
    # C4 (n=512): its bench K=5 iterations, 4 problems (the
    # blocked kernel's configuration)
    # C2: its bench K=8 iterations (the trajectory gates cover every iteration the bench times)
    for cfg, count, iters in ((C0B, 4, 6), (C1, 8, 4), (C2, 8, 8), (C4, 4, 5)):
        d = O.generate(cfg.cones, count, cfg.n, cfg.m, cfg.k, cfg.seed)
        for p in range(count):
            c = d["c"][p * cfg.n:(p + 1) * cfg.n]
            A = d["A"][p * cfg.m * cfg.n:(p + 1) * cfg.m * cfg.n].reshape(cfg.n, cfg.m).T
            b = d["b"][p * cfg.m:(p + 1) * cfg.m]
            G = d["G"][p * cfg.k * cfg.n:(p + 1) * cfg.k * cfg.n].reshape(cfg.n, cfg.k).T
            h = d["h"][p * cfg.k:(p + 1) * cfg.k]
            out["cases"].append(case(f"{cfg.name}#{p}", [tuple(t) for t in cfg.cones], c, A, b, G, h, iters,
                                     {"config": cfg.name, "seed": cfg.seed, "problem": p}))
    path = os.path.join(HERE, "trajectories.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print(f"wrote {path}: {len(out['cases'])} cases, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
