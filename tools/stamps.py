"""Phase breakdown (shader-clock cycles per problem-iteration per wave) from the
diagnostic build libsocp_diag.so (SOCP_STAMPS).  Diagnostic only: its run time
is not a benchmark number (stamps serialise the waits)."""
import os, sys, time
HERE = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("SOCP_AMD_LIB", os.path.join(HERE, "..", "socp.jl_amd", "lib", "libsocp_diag.so"))
sys.path.insert(0, os.path.join(HERE, "..", "socp.jl_amd"))
import torch
import socp_amd as S
from socp_amd import _lib
from socp_amd.configs import CONFIGS
names = ["load", "scaling", "resid", "U", "SYRK", "sweepH", "schur", "solve", "step", "vop", "store", "other"]
RUNS = {"C2": (8192, 8), "C1": (4096, 3), "C4": (256, 3)}
for cname in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["C2", "C1"]):
    B, K = RUNS[cname]
    cfg = CONFIGS[cname]
    ctx = S.default_context()
    c, A, b, G, h = S.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
    sing = torch.zeros(B, dtype=torch.uint8, device="cuda")
    buf = torch.zeros(24, dtype=torch.int64, device="cuda")
    _lib.load().socp_debug_set_stamps(_lib.ptr(buf))
    out = S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, c, A, b, G, h, sing, maxit=K, tol=0.0)
    ctx.sync(); buf.zero_()
    out = S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, c, A, b, G, h, sing, maxit=K, tol=0.0)
    ctx.sync()
    v = buf.cpu().numpy().astype(float)
    iters = v[12]
    tot = v[:12].sum() + v[13:24].sum()
    print(f"== {cname} B={B} K={K} kernel {ctx.last_kernel_ms():.2f} ms, iters {iters:.0f}, cycles/problem-iter {tot/iters:.0f}")
    for nm, x in zip(names, v[:12]):
        print(f"   {nm:8s} {x/iters:9.0f} cyc/it  {100*x/tot:5.1f}%")
    if cname == "C4":
        subs = ["sw:catchup", "sw:pivots", "sw:writebk", "sw:final", "finalize", "gemv_Gt", "symv", "gemv_G"]
    else:
        subs = ["sw:fac0", "sw:fac+ops", "sw:T+Y", "sw:last", "s:Gt", "s:symvH", "s:A,S", "s:ALt", "v:headred",
            "v:tailred1", "v:tailred2"]
    for nm, x in zip(subs, v[13:24]):
        if x:
            print(f"   {nm:9s} {x/iters:8.0f} cyc/it  {100*x/tot:5.1f}%")
