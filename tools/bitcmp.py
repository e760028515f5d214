"""Writes (or compares against) the C4 solution of a small batch: bit-identity
check between two libsocp builds.  usage: bitcmp.py save|compare FILE"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "socp.jl_amd"))
import socp_amd as S  # noqa: E402
from socp_amd.configs import C4  # noqa: E402

mode, path = sys.argv[1], sys.argv[2]
B = 32
c, A, b, G, h = S.generate(C4.cones, B, C4.n, C4.m, C4.k, C4.seed)
import torch  # noqa: E402
sing = torch.zeros(B, dtype=torch.uint8, device=G.device)
out = S.batch_solve(C4.cones, C4.n, C4.m, C4.k, c, A, b, G, h, sing, maxit=5, tol=0.0)
S.default_context().sync()
x = np.concatenate([out[k].cpu().numpy().ravel() for k in ("x", "y", "z", "s")])
if mode == "save":
    with open(path, "wb") as f:
        f.write(x.tobytes())
else:
    ref = np.frombuffer(open(path, "rb").read(), dtype=np.float64)
    diff = int((ref.view(np.uint64) != x.view(np.uint64)).sum())
    print(f"{diff} of {x.size} values differ bitwise; max rel {np.max(np.abs(ref - x)) / np.max(np.abs(ref)):.3e}")
