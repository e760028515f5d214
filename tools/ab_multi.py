"""A/B of several libsocp builds in ONE process (tuning tool, not a test).

  python tools/ab_multi.py C2 8 lib/a/libsocp.so lib/b/libsocp.so ...

Each library is dlopen'ed separately (after torch, so all share torch's HIP
runtime); the config's batch is generated once on the device by the first
library, then every library solves it (fixed-K, device pointers) in
interleaved rounds.  Prints per library the median / min solver-kernel time
(HIP events, socp_last_kernel_ms) and the largest relative difference of x
from the first library's result."""
import ctypes as C
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "socp.jl_amd"))
from socp_amd import _lib  # noqa: E402
from socp_amd.configs import CONFIGS  # noqa: E402

cfg = CONFIGS[sys.argv[1]]
reps = int(sys.argv[2])
paths = sys.argv[3:]
if os.environ.get("AB_SHAPE"):  # probe shapes: "n,m,k" with POC(0, k/2) + SOC(k/2, k - k/2)
    import dataclasses
    n_, m_, k_ = map(int, os.environ["AB_SHAPE"].split(","))
    cfg = dataclasses.replace(cfg, n=n_, m=m_, k=k_, cones=((0, 0, k_ // 2), (1, k_ // 2, k_ - k_ // 2)))
B, n, m, k = cfg.batch, cfg.n, cfg.m, cfg.k
if os.environ.get("AB_BATCH"):
    B = int(os.environ["AB_BATCH"])
K = int(os.environ.get("AB_K", cfg.fixed_k))
libs = []
for p in paths:
    L = C.CDLL(os.path.abspath(p), mode=C.RTLD_LOCAL)
    vp = C.c_void_p
    common = [vp, C.POINTER(_lib.Dims), vp, vp, vp]
    L.socp_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.socp_ctx_sync.argtypes = [vp]
    L.socp_batch_solve.argtypes = common + [vp] * 5 + [vp, C.POINTER(_lib.Params)] + [vp] * 4 + [vp, vp]
    L.socp_generate.argtypes = common + [C.c_uint64, C.c_int64] + [vp] * 5
    L.socp_last_kernel_ms.argtypes = [vp, C.POINTER(C.c_float)]
    L.socp_last_error.restype = C.c_char_p
    h = C.c_void_p()
    assert L.socp_ctx_create(0, C.byref(h)) == 0
    libs.append((p, L, h))

dev = torch.device("cuda", 0)
kind = (C.c_int32 * len(cfg.cones))(*[c[0] for c in cfg.cones])
offs = (C.c_int32 * len(cfg.cones))(*[c[1] for c in cfg.cones])
dim = (C.c_int32 * len(cfg.cones))(*[c[2] for c in cfg.cones])
dims = _lib.Dims(B, n, m, k, len(cfg.cones))
f64 = dict(dtype=torch.float64, device=dev)
c, A, b, G, h = (torch.empty(B * q, **f64) for q in (n, m * n, m, k * n, k))
P0 = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
L0, h0 = libs[0][1], libs[0][2]
assert L0.socp_generate(h0, C.byref(dims), kind, offs, dim, cfg.seed, 0, *map(P0, (c, A, b, G, h))) == 0
L0.socp_ctx_sync(h0)
sing = torch.zeros(B, dtype=torch.uint8, device=dev)
params = _lib.default_params(maxit=K, tol=0.0, flags=_lib.F_DEVICE_PTRS)
outs = []
for _ in libs:
    outs.append(dict(x=torch.empty(B * n, **f64), y=torch.empty(B * max(m, 1), **f64), z=torch.empty(B * k, **f64),
                     s=torch.empty(B * k, **f64), it=torch.empty(B, dtype=torch.int32, device=dev),
                     st=torch.empty(B, dtype=torch.int32, device=dev)))
times = [[] for _ in libs]
for r in range(reps + 1):
    for i, (p, L, hh) in enumerate(libs):
        o = outs[i]
        rc = L.socp_batch_solve(hh, C.byref(dims), kind, offs, dim, *map(P0, (c, A, b, G, h)), P0(sing),
                                C.byref(params), *map(P0, (o["x"], o["y"], o["z"], o["s"], o["it"], o["st"])))
        if rc:
            raise RuntimeError(f"{p}: {rc} {L.socp_last_error().decode()}")
        L.socp_ctx_sync(hh)
        ms = C.c_float()
        L.socp_last_kernel_ms(hh, C.byref(ms))
        if r:
            times[i].append(ms.value)
x0 = outs[0]["x"].view(B, n)
for i, (p, _, _) in enumerate(libs):
    t = sorted(times[i])
    x = outs[i]["x"].view(B, n)
    rel = ((x - x0).norm(dim=1) / x0.norm(dim=1).clamp_min(1e-300)).max().item()
    st = torch.bincount(outs[i]["st"].long(), minlength=5).tolist()
    print(f"{sys.argv[1]} {os.path.relpath(p)}: median {t[len(t)//2]:.3f} ms  min {t[0]:.3f} ms  "
          f"max rel dx vs first {rel:.2e}  status {st}  iters {int(outs[i]['it'].sum())}", flush=True)
