# SocpHip.jl — Julia-side binding of libsocp (include/socp.h) for BenChung/Socp.jl.
#
# Drop-in for the dense path: `HipDenseSolver <: KKTSolver{Scaling}` plugs into
# the reference's `SolverState(prob, solver)` / `solve_socp(prob, ss)`
# (solver.jl:22,40), and `solve_socp_batched` runs a whole batch of problems
# (same dims and cones) in one device call.  All arithmetic happens in the HIP
# kernels of libsocp.so; this file only marshals arrays through `ccall`.
#
# Usage (inside module Socp, after `include("densesolver.jl")`):
#     include(joinpath(SOCP_AMD_DIR, "julia", "SocpHip.jl"))
#     ss = SolverState(prob, HipDenseSolver(prob))
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
mutable struct HipDenseSolver <: KKTSolver{Scaling}
    A::Matrix{Float64}
    G::Matrix{Float64}
    s::Vector{Float64}
    z::Vector{Float64}
end
HipDenseSolver(pr::Problem) = HipDenseSolver(Matrix(pr.A), Matrix(pr.G), zeros(pr.k), zeros(pr.k))

# setup_iter(::DenseSolver) (densesolver.jl:41-52): the factorisation is fused
# with the solve on the device; record the iterate it applies to.
function setup_iter(ss::HipDenseSolver, pr::Problem{C,n,m,k,sing}, s::State, scaling::Scaling) where {C,n,m,k,sing}
    copyto!(ss.s, s.s)
    copyto!(ss.z, s.z)
    return nothing
end

# solve_kkt(::DenseSolver) (densesolver.jl:54-90): one socp_batch_kkt_solve with batch 1.
function solve_kkt(ss::HipDenseSolver, pr::Problem{C,n,m,k,sing}, s::State, scaling::Scaling,
                   dx::Vector{Float64}, dy::Vector{Float64}, dz::Vector{Float64}, ds::Vector{Float64},
                   cx::Vector{Float64}, cy::Vector{Float64}, cz::Vector{Float64}, cs::Vector{Float64}) where {C,n,m,k,sing}
    kind, offs, dim = cone_arrays(pr.cones)
    dims = Ref(SocpDims(1, n, m, k, length(pr.cones)))
    singv = UInt8[sing ? 1 : 0]
    st = Int32[0]
    rc = ccall((:socp_batch_kkt_solve, libsocp), Cint,
               (Ptr{Cvoid}, Ref{SocpDims}, Ptr{Int32}, Ptr{Int32}, Ptr{Int32},
                Ptr{Float64}, Ptr{Float64}, Ptr{UInt8}, Ptr{Float64}, Ptr{Float64},
                Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Int32),
               socp_ctx(), dims, kind, offs, dim, ss.A, ss.G, singv, ss.s, ss.z,
               dx, dy, dz, ds, cx, cy, cz, cs, st, Int32(0))
    socp_check(rc)
    socp_throw(st[1])
    return nothing
end

# ------------------------------------------------------------ batched solve
"""
    solve_socp_batched(problems; maxit=40, tol=1e-5) -> (states, iters, status)

`solve_socp` (solver.jl:40-153) for every problem of a vector sharing
`n, m, k` and the cone tuple, in one device call.  Failures are reported per
problem in `status` (0 converged, 1 maxit, 2/3 PosDef, 4 domain) instead of
throwing, so one bad problem does not abort the batch.
"""
function solve_socp_batched(problems::AbstractVector{<:Problem}; maxit=40, tol=1e-5)
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
    params = Ref(SocpParams(maxit, 3, tol, 0.99, 1e-10, 0, 0))
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

# ------------------------------------------------------- multi-GPU gather
# One process per GPU (e.g. under MPI.jl); problems shard by contiguous global
# index and the only collective is the RCCL all-gather of (status, iters)
# (include/socp.h: socp_comm_*, socp_allgather_status).  Rank 0 makes the id,
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

# Example (MPI.jl):
#   id = MPI.Comm_rank(comm) == 0 ? socp_comm_unique_id() : zeros(UInt8, SOCP_COMM_ID_BYTES)
#   MPI.Bcast!(id, 0, comm)
#   c = socp_comm_init(MPI.Comm_size(comm), MPI.Comm_rank(comm), id)
