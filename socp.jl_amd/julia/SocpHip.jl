# SocpHip.jl — Julia-side binding of libsocp (include/socp.h) for BenChung/Socp.jl.
#
# Drop-in for the dense path: `HipDenseSolver <: KKTSolver{HipScaling}` plugs into
# the reference's `SolverState(prob, solver)` / `solve_socp(prob, ss)`
# (solver.jl:22,40), and `solve_socp_batched` runs a whole batch of problems
# (same dims and cones) in one device call.  All arithmetic happens in the HIP
# kernels of libsocp.so; this file only marshals arrays through `ccall`.
#
# Usage (inside module Socp, after `include("densesolver.jl")`):
#     include(joinpath(SOCP_AMD_DIR, "julia", "SocpHip.jl"))
#     ss = SolverState(prob, HipDenseSolver(prob))           # scaling type: HipScaling
#     setup_iter(ss.solver, prob, state, scaling)            # densesolver.jl:41
#     solve_kkt(ss.solver, prob, state, scaling, dx,dy,dz,ds, cx,cy,cz,cs)  # densesolver.jl:54
#     xs = solve_socp_batched(problems)                       # batched solve_socp
#
# Not executed in this repository's CI (no Julia in the image); the C ABI it
# binds is exercised by tests/ through Python ctypes with the same argument
# meaning.

const libsocp = get(ENV, "SOCP_AMD_LIB",
                    joinpath(@__DIR__, "..", "lib", "libsocp.so"))

const SOCP_F_DEVICE_PTRS = Int32(1)
const SOCP_F_WARM_START = Int32(2)
const SOCP_F_EXPLICIT_INVERSE = Int32(8)   # Li = H^-1 formed, the reference's op order (densesolver.jl:48)

struct SocpDims
    batch::Int64
    n::Int32
    m::Int32
    k::Int32
    ncones::Int32
end

struct SocpParams
    maxit::Int32
    sigma_exp::Int32
    tol::Float64
    step::Float64
    init_eps::Float64
    flags::Int32
    reserved::Int32
end
SocpParams() = SocpParams(40, 3, 1e-5, 0.99, 1e-10, 0, 0)   # solver.jl:105,122,133,146,91

const _ctx = Ref{Ptr{Cvoid}}(C_NULL)
function socp_ctx()
    if _ctx[] == C_NULL
        h = Ref{Ptr{Cvoid}}(C_NULL)
        rc = ccall((:socp_ctx_create, libsocp), Cint, (Cint, Ptr{Ptr{Cvoid}}), 0, h)
        rc == 0 || error("socp_ctx_create: ", unsafe_string(ccall((:socp_last_error, libsocp), Cstring, ())))
        _ctx[] = h[]
    end
    return _ctx[]
end

socp_check(rc) = rc == 0 || error("libsocp: ", unsafe_string(ccall((:socp_last_error, libsocp), Cstring, ())))

cone_kind(::POC) = Int32(0)
cone_kind(::SOC) = Int32(1)
cone_arrays(cones) = (Int32[cone_kind(c) for c in cones], Int32[c.offs for c in cones],
                      Int32[conedim(c) for c in cones])

# status codes of include/socp.h -> the exceptions the reference throws
function socp_throw(st)
    st == 2 && throw(PosDefException(1))          # cholesky!(H), densesolver.jl:47
    st == 3 && throw(PosDefException(1))          # cholesky!(S), densesolver.jl:51
    st == 4 && throw(DomainError(-1.0, "sqrt of a negative number"))
    return nothing
end

# --------------------------------------------------------------- plugin
# HipDenseSolver mirrors DenseSolver's life cycle on the device (include/socp.h,
# socp_dense_*): construction copies A and G into a one-problem handle once
# (densesolver.jl:19-38), setup_iter factors into the handle's device record
# (:41-52), solve_kkt solves against it (:54-90) -- the solver calls it twice per
# iteration (solver.jl:127,141) -- moving only n+m+2k doubles.

# HipScaling: the lightweight AbstractScaling of the plugin.  SolverState is
# generic in its scaling type (solver.jl:1-2,22-23: S(pr) for KKTSolver{S}), and
# the driver loop reads only scaling.l and calls scale!/iscale! (solver.jl:107,
# 128-129,143-144), which need the per-cone wb and mu -- O(k) data.  The dense
# W, W^-1 and the k^3 iW*iW' product of the reference's Scaling
# (scalings.jl:1-20,108) are never formed on the host: the device computes its
# own NT scaling from (s, z) inside setup_iter.
struct HipScaling <: AbstractScaling
    l::Vector{Float64}     # lambda = W z
    mu::Vector{Float64}    # per cone: sqrt(||s||_J / ||z||_J) (1 for POC)
    wbs::Vector{Float64}   # POC: sqrt(s/z); SOC: the unit NT vector wb
end
HipScaling(p::Problem) = HipScaling(zeros(p.k), zeros(length(p.cones)), zeros(p.k))

function hip_scaling!(c::POC, ci, sc::HipScaling, s, z)
    for i in cti(c, 1):cti(c, conedim(c))
        sc.wbs[i] = sqrt(s[i] / z[i])
        sc.l[i] = sqrt(s[i] * z[i])
    end
end

# NT scaling of one second-order cone (scalings.jl:32-99) restated on vectors:
# normalised s and z, gamma, wb, mu and lambda, no matrices.
function hip_scaling!(c::SOC, ci, sc::HipScaling, s, z)
    o, d = cti(c, 1), conedim(c)
    jz, js = z[o]^2, s[o]^2
    for i in o+1:o+d-1
        jz -= z[i] * z[i]
        js -= s[i] * s[i]
    end
    nz, ns = sqrt(jz), sqrt(js)          # DomainError off the cone, like the reference
    fz, fs = 1 / nz, 1 / ns
    dot = 0.0
    for i in o:o+d-1
        dot += (z[i] * fz) * (s[i] * fs)
    end
    gamma = sqrt((1 + dot) / 2)
    g2 = 1 / (2 * gamma)
    sc.wbs[o] = (s[o] * fs + z[o] * fz) * g2
    for i in o+1:o+d-1
        sc.wbs[i] = (s[i] * fs - z[i] * fz) * g2
    end
    sc.mu[ci] = sqrt(ns / nz)
    z0, s0 = z[o] * fz, s[o] * fs
    rt = sqrt(ns * nz)
    mult = rt / (z0 + s0 + 2 * gamma)
    for i in o+1:o+d-1
        sc.l[i] = ((s[i] * fs) * (gamma + z0) + (z[i] * fz) * (gamma + s0)) * mult
    end
    sc.l[o] = gamma * rt
end

function compute_scaling(cones::Tuple{Vararg{Cone}}, sc::HipScaling, s, z)
    for (ci, c) in enumerate(cones)
        c isa POC && (sc.mu[ci] = 1.0)
        hip_scaling!(c, ci, sc, s, z)
    end
    return sc
end
# W s and W^-1 s (scalings.jl:112-160): the per-cone methods read only wbs and mu
function scale!(cones::Tuple{Vararg{Cone}}, sc::HipScaling, s, op)
    for (ci, c) in enumerate(cones)
        scale!(c, ci, sc, s, op)
    end
end
function iscale!(cones::Tuple{Vararg{Cone}}, sc::HipScaling, s, op)
    for (ci, c) in enumerate(cones)
        iscale!(c, ci, sc, s, op)
    end
end

mutable struct HipDenseSolver <: KKTSolver{HipScaling}
    handle::Ptr{Cvoid}
    status::Vector{Int32}
    # explicit_inverse=true: SOCP_F_EXPLICIT_INVERSE, Li = H^-1 formed as densesolver.jl:48 does
    function HipDenseSolver(pr::Problem{C,n,m,k,sing}; explicit_inverse::Bool=false) where {C,n,m,k,sing}
        kind, offs, dim = cone_arrays(pr.cones)
        dims = Ref(SocpDims(1, n, m, k, length(pr.cones)))
        A = Matrix{Float64}(pr.A)   # column-major m x n, as include/socp.h lays it out
        G = Matrix{Float64}(pr.G)
        singv = UInt8[sing ? 1 : 0]
        h = Ref{Ptr{Cvoid}}(C_NULL)
        socp_check(ccall((:socp_dense_create, libsocp), Cint,
                         (Ptr{Cvoid}, Ref{SocpDims}, Ptr{Int32}, Ptr{Int32}, Ptr{Int32},
                          Ptr{Float64}, Ptr{Float64}, Ptr{UInt8}, Int32, Ptr{Ptr{Cvoid}}),
                         socp_ctx(), dims, kind, offs, dim, A, G, singv,
                         explicit_inverse ? SOCP_F_EXPLICIT_INVERSE : Int32(0), h))
        ss = new(h[], Int32[0])
        finalizer(ss) do x
            x.handle == C_NULL || ccall((:socp_dense_destroy, libsocp), Cint, (Ptr{Cvoid},), x.handle)
            x.handle = C_NULL
        end
        return ss
    end
end

# setup_iter(::DenseSolver) (densesolver.jl:41-52): scaling of (s, z), H and its
# factorisation, kept in the handle on the device: by default the Cholesky
# factor L of H, Z = L^-1 A' and S^-1 (S = Z'Z = A H^-1 A'; H^-1 is never
# formed), or -- with SOCP_F_EXPLICIT_INVERSE at create, and on m > 16 register
# shapes -- Li = H^-1, A Li and S^-1 as densesolver.jl:48-51 do.
function setup_iter(ss::HipDenseSolver, pr::Problem{C,n,m,k,sing}, s::State, scaling::HipScaling) where {C,n,m,k,sing}
    socp_check(ccall((:socp_dense_setup_iter, libsocp), Cint,
                     (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}), ss.handle, s.s, s.z, ss.status))
    socp_throw(ss.status[1])
    return nothing
end

# solve_kkt(::DenseSolver) (densesolver.jl:54-90) against the last setup_iter.
function solve_kkt(ss::HipDenseSolver, pr::Problem{C,n,m,k,sing}, s::State, scaling::HipScaling,
                   dx::Vector{Float64}, dy::Vector{Float64}, dz::Vector{Float64}, ds::Vector{Float64},
                   cx::Vector{Float64}, cy::Vector{Float64}, cz::Vector{Float64}, cs::Vector{Float64}) where {C,n,m,k,sing}
    socp_check(ccall((:socp_dense_solve_kkt, libsocp), Cint,
                     (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                      Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}),
                     ss.handle, dx, dy, dz, ds, cx, cy, cz, cs, ss.status))
    socp_throw(ss.status[1])
    return nothing
end

# ---------------------------------------------------- rank-update plugin
# HipSqrSolver replaces SparseSolver (spsolver.jl:1-130) -- the solver the
# reference's own tests and MOI wrapper run -- on the device (include/socp.h,
# socp_sqr_*): SqrScaling's W^-2 = D + uu' - vv' (sqrscalings.jl:66-139), the
# factor of G'DG (+A'A), one rank-1 update and one downdate per SOC cone
# (modify_factors!, sqrscalings.jl:160-194) and the factor of S, all inside
# setup_iter; solve_kkt by triangular solves.  Its scaling type is the same
# HipScaling: SqrScaling's l, wbs, mu equal Scaling's (runtests.jl:58-60,71-73),
# and the driver loop reads nothing else.  Usage:
#     ss = SolverState(prob, HipSqrSolver(prob)); solve_socp(prob, ss)
mutable struct HipSqrSolver <: KKTSolver{HipScaling}
    handle::Ptr{Cvoid}
    status::Vector{Int32}
    function HipSqrSolver(pr::Problem{C,n,m,k,sing}) where {C,n,m,k,sing}
        kind, offs, dim = cone_arrays(pr.cones)
        dims = Ref(SocpDims(1, n, m, k, length(pr.cones)))
        A = Matrix{Float64}(pr.A)
        G = Matrix{Float64}(pr.G)
        singv = UInt8[sing ? 1 : 0]
        h = Ref{Ptr{Cvoid}}(C_NULL)
        socp_check(ccall((:socp_sqr_create, libsocp), Cint,
                         (Ptr{Cvoid}, Ref{SocpDims}, Ptr{Int32}, Ptr{Int32}, Ptr{Int32},
                          Ptr{Float64}, Ptr{Float64}, Ptr{UInt8}, Int32, Ptr{Ptr{Cvoid}}),
                         socp_ctx(), dims, kind, offs, dim, A, G, singv, Int32(0), h))
        ss = new(h[], Int32[0])
        finalizer(ss) do x
            x.handle == C_NULL || ccall((:socp_sqr_destroy, libsocp), Cint, (Ptr{Cvoid},), x.handle)
            x.handle = C_NULL
        end
        return ss
    end
end

function setup_iter(ss::HipSqrSolver, pr::Problem{C,n,m,k,sing}, s::State, scaling::HipScaling) where {C,n,m,k,sing}
    socp_check(ccall((:socp_sqr_setup_iter, libsocp), Cint,
                     (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}), ss.handle, s.s, s.z, ss.status))
    socp_throw(ss.status[1])
    return nothing
end

function solve_kkt(ss::HipSqrSolver, pr::Problem{C,n,m,k,sing}, s::State, scaling::HipScaling,
                   dx::Vector{Float64}, dy::Vector{Float64}, dz::Vector{Float64}, ds::Vector{Float64},
                   cx::Vector{Float64}, cy::Vector{Float64}, cz::Vector{Float64}, cs::Vector{Float64}) where {C,n,m,k,sing}
    socp_check(ccall((:socp_sqr_solve_kkt, libsocp), Cint,
                     (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                      Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}),
                     ss.handle, dx, dy, dz, ds, cx, cy, cz, cs, ss.status))
    socp_throw(ss.status[1])
    return nothing
end

# ------------------------------------------------------------ batched solve
"""
    solve_socp_batched(problems; maxit=40, tol=1e-5, explicit_inverse=false) -> (states, iters, status)

`solve_socp` (solver.jl:40-153) for every problem of a vector sharing
`n, m, k` and the cone tuple, in one device call.  Failures are reported per
problem in `status` (0 converged, 1 maxit, 2/3 PosDef, 4 domain) instead of
throwing, so one bad problem does not abort the batch.
"""
function solve_socp_batched(problems::AbstractVector{<:Problem}; maxit=40, tol=1e-5, explicit_inverse::Bool=false)
    p0 = problems[1]
    n, m, k = p0.n, p0.m, p0.k
    B = length(problems)
    kind, offs, dim = cone_arrays(p0.cones)
    c = reduce(vcat, [p.c for p in problems])
    A = reduce(vcat, [vec(Matrix(p.A)) for p in problems])     # column-major per problem
    b = reduce(vcat, [p.b for p in problems])
    G = reduce(vcat, [vec(Matrix(p.G)) for p in problems])
    h = reduce(vcat, [p.h for p in problems])
    sing = UInt8[typeof(p).parameters[5] ? 1 : 0 for p in problems]
    x, y, z, s = zeros(B * n), zeros(B * m), zeros(B * k), zeros(B * k)
    iters, status = zeros(Int32, B), zeros(Int32, B)
    params = Ref(SocpParams(maxit, 3, tol, 0.99, 1e-10, explicit_inverse ? SOCP_F_EXPLICIT_INVERSE : Int32(0), 0))
    dims = Ref(SocpDims(B, n, m, k, length(p0.cones)))
    rc = ccall((:socp_batch_solve, libsocp), Cint,
               (Ptr{Cvoid}, Ref{SocpDims}, Ptr{Int32}, Ptr{Int32}, Ptr{Int32},
                Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{UInt8},
                Ref{SocpParams}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                Ptr{Int32}, Ptr{Int32}),
               socp_ctx(), dims, kind, offs, dim, c, A, b, G, h, sing, params,
               x, y, z, s, iters, status)
    socp_check(rc)
    states = [State(problems[i], x[(i-1)*n+1:i*n], y[(i-1)*m+1:i*m], z[(i-1)*k+1:i*k], s[(i-1)*k+1:i*k])
              for i in 1:B]
    return states, iters, status
end

"""
    solve_socp_batched_sqr(problems; maxit=40, tol=1e-5) -> (states, iters, status)

The same batch through the rank-update plugin: `solve_socp(prob,
SolverState(prob, SparseSolver(prob)))` for every problem, the reference's own
tested configuration, as one device solve (`socp_sqr_create` +
`socp_sqr_solve_socp`; failures per problem, no throw).
"""
function solve_socp_batched_sqr(problems::AbstractVector{<:Problem}; maxit=40, tol=1e-5)
    p0 = problems[1]
    n, m, k = p0.n, p0.m, p0.k
    B = length(problems)
    kind, offs, dim = cone_arrays(p0.cones)
    c = reduce(vcat, [p.c for p in problems])
    A = reduce(vcat, [vec(Matrix(p.A)) for p in problems])
    b = reduce(vcat, [p.b for p in problems])
    G = reduce(vcat, [vec(Matrix(p.G)) for p in problems])
    h = reduce(vcat, [p.h for p in problems])
    sing = UInt8[typeof(p).parameters[5] ? 1 : 0 for p in problems]
    dims = Ref(SocpDims(B, n, m, k, length(p0.cones)))
    hd = Ref{Ptr{Cvoid}}(C_NULL)
    socp_check(ccall((:socp_sqr_create, libsocp), Cint,
                     (Ptr{Cvoid}, Ref{SocpDims}, Ptr{Int32}, Ptr{Int32}, Ptr{Int32},
                      Ptr{Float64}, Ptr{Float64}, Ptr{UInt8}, Int32, Ptr{Ptr{Cvoid}}),
                     socp_ctx(), dims, kind, offs, dim, A, G, sing, Int32(0), hd))
    x, y, z, s = zeros(B * n), zeros(B * m), zeros(B * k), zeros(B * k)
    iters, status = zeros(Int32, B), zeros(Int32, B)
    params = Ref(SocpParams(maxit, 3, tol, 0.99, 1e-10, 0, 0))
    try
        socp_check(ccall((:socp_sqr_solve_socp, libsocp), Cint,
                         (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ref{SocpParams},
                          Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32},
                          Ptr{Float64}),
                         hd[], c, b, h, params, x, y, z, s, iters, status, C_NULL))
    finally
        ccall((:socp_sqr_destroy, libsocp), Cint, (Ptr{Cvoid},), hd[])
    end
    states = [State(problems[i], x[(i-1)*n+1:i*n], y[(i-1)*m+1:i*m], z[(i-1)*k+1:i*k], s[(i-1)*k+1:i*k])
              for i in 1:B]
    return states, iters, status
end

# ------------------------------------------------------- multi-GPU gather
# One process per GPU (e.g. under MPI.jl); problems shard by contiguous global
# index and the only collective is the RCCL all-gather of each problem's
# 32-byte outcome record (include/socp.h: socp_comm_*, socp_allgather_outcomes;
# socp_allgather_status gathers only (status, iters)).  Rank 0 makes the id,
# the host broadcasts it (MPI.Bcast! below is the usual way).
const SOCP_COMM_ID_BYTES = 128

function socp_comm_unique_id()
    id = zeros(UInt8, SOCP_COMM_ID_BYTES)
    socp_check(ccall((:socp_comm_unique_id, libsocp), Cint, (Ptr{UInt8},), id))
    return id
end

function socp_comm_init(nranks::Integer, rank::Integer, id::Vector{UInt8})
    h = Ref{Ptr{Cvoid}}(C_NULL)
    socp_check(ccall((:socp_comm_init, libsocp), Cint,
                     (Ptr{Cvoid}, Cint, Cint, Ptr{UInt8}, Ptr{Ptr{Cvoid}}),
                     socp_ctx(), nranks, rank, id, h))
    return h[]
end

socp_comm_destroy(comm::Ptr{Cvoid}) = ccall((:socp_comm_destroy, libsocp), Cint, (Ptr{Cvoid},), comm)

# status, iters, out: device pointers (out holds nranks * B * 2 Int32, rank-major)
function socp_allgather_status(comm::Ptr{Cvoid}, B::Integer, status::Ptr{Int32}, iters::Ptr{Int32},
                               out::Ptr{Int32})
    socp_check(ccall((:socp_allgather_status, libsocp), Cint,
                     (Ptr{Cvoid}, Int64, Ptr{Int32}, Ptr{Int32}, Ptr{Int32}), comm, B, status, iters, out))
    socp_check(ccall((:socp_ctx_sync, libsocp), Cint, (Ptr{Cvoid},), socp_ctx()))
    return nothing
end

# The 32-byte per-problem outcome record of include/socp.h (socp_outcome): the
# exit-test quantities of solver.jl:109-122 at the returned iterate.
struct SocpOutcome
    status::Int32
    iters::Int32
    res_dual::Float64    # ||A'y + G'z + c||
    res_primal::Float64  # ||Ax - b||
    gap::Float64         # z's
end

# status, iters (B Int32 each), res (3B Float64: ||rd||, ||rp||, z's per problem,
# as socp_batch_solve_ex writes them; C_NULL gives NaN residuals) and out
# (nranks * B SocpOutcome, rank-major: out[r*B + p] is rank r's problem p) are
# device pointers; returns after the gather has completed.
function socp_allgather_outcomes(comm::Ptr{Cvoid}, B::Integer, status::Ptr{Int32}, iters::Ptr{Int32},
                                 res::Ptr{Float64}, out::Ptr{SocpOutcome})
    socp_check(ccall((:socp_allgather_outcomes, libsocp), Cint,
                     (Ptr{Cvoid}, Int64, Ptr{Int32}, Ptr{Int32}, Ptr{Float64}, Ptr{SocpOutcome}),
                     comm, B, status, iters, res, out))
    socp_check(ccall((:socp_ctx_sync, libsocp), Cint, (Ptr{Cvoid},), socp_ctx()))
    return nothing
end

# Example (MPI.jl):
#   id = MPI.Comm_rank(comm) == 0 ? socp_comm_unique_id() : zeros(UInt8, SOCP_COMM_ID_BYTES)
#   MPI.Bcast!(id, 0, comm)
#   c = socp_comm_init(MPI.Comm_size(comm), MPI.Comm_rank(comm), id)
