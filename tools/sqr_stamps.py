"""Phase breakdown of the rank-update setup kernel (socp_sqr_setup_kernel):
shader-clock cycles per problem per workgroup from the diagnostic build
libsocp_diag.so.  Diagnostic only."""
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("SOCP_AMD_LIB", os.path.join(HERE, "..", "socp.jl_amd", "lib", "libsocp_diag.so"))
sys.path.insert(0, os.path.join(HERE, "..", "socp.jl_amd"))
import torch
import socp_amd as S
from socp_amd import _lib
from socp_amd.configs import CONFIGS
names = ["load+scaling", "H=G'DG", "chol(H)", "rank-1 mods", "L^-1 A'", "S+chol(S)", "record"]
cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C2"]
B = 8192
ctx = S.default_context()
c, A, b, G, h = S.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed)
sing = torch.zeros(B, dtype=torch.uint8, device="cuda")
out = S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, c, A, b, G, h, sing, maxit=3, tol=0.0)
ctx.sync()
hd = S.SqrHandle(cfg.cones, cfg.n, cfg.m, cfg.k, A, G, sing)
buf = torch.zeros(24, dtype=torch.int64, device="cuda")
_lib.load().socp_debug_set_stamps(_lib.ptr(buf))
hd.setup_iter(out["s"], out["z"])
ctx.sync()
buf.zero_()
hd.setup_iter(out["s"], out["z"])
ctx.sync()
ms = ctx.last_kernel_ms()
v = buf.cpu().numpy().astype(float)
tot = v[:7].sum()
print(f"== {cfg.name} B={B} setup kernel {ms:.3f} ms, cycles/problem {tot / B:.0f}")
for nm, x in zip(names, v[:7]):
    print(f"   {nm:14s} {x / B:9.0f} cyc  {100 * x / tot:5.1f}%")
buf.zero_()
r = [torch.randn(B * q, dtype=torch.float64, device="cuda") for q in (cfg.n, cfg.m, cfg.k, cfg.k)]
hd.solve_kkt(*r)
ctx.sync()
ms = ctx.last_kernel_ms()
v = buf.cpu().numpy().astype(float)
sn = ["load+cone head", "G'k1", "fwd #1", "bwd #1", "A,S,A'", "fwd+bwd #2", "Gcx+cone tail"]
tot = v[8:15].sum()
print(f"== solve kernel {ms:.3f} ms, cycles/problem {tot / B:.0f}")
for nm, x in zip(sn, v[8:15]):
    print(f"   {nm:14s} {x / B:9.0f} cyc  {100 * x / tot:5.1f}%")
