# SocpHipMOI.jl — routes the reference's MathOptInterface adapter (src/moi.jl)
# to the HIP dense path (SURVEY.md §8(f) row 2).  Include inside module Socp
# after moi.jl and SocpHip.jl:
#     include(joinpath(SOCP_AMD_DIR, "julia", "SocpHipMOI.jl"))
#
# `HipOptimizer <: MOI.AbstractOptimizer` WRAPS the reference `Optimizer`
# (moi.jl:59-67): model loading (copy_to, the allocate/load API,
# moi.jl:95-197) runs on the wrapped object unchanged, and this file adds
# methods only for HipOptimizer -- no method of moi.jl is redefined (Julia
# >= 1.10 rejects overwriting a method during precompilation).  Use
#     MOI.instantiate(() -> Socp.HipOptimizer(maxit=40); with_bridge_type=Float64)
# where the reference example uses Socp.Optimizer (moi.jl:229).
#
# What HipOptimizer's optimize! / getters do differently from moi.jl (each
# cites the line whose behaviour it replaces):
#   * solve_socp gets SolverState(prob, HipDenseSolver(prob)) -- moi.jl:222
#     passes a SparseSolver where solve_socp (solver.jl:40) expects a SolverState;
#   * cones are a Tuple (Problem's type parameter C) -- moi.jl:215 builds a
#     Vector{Cone}, which Problem (Socp.jl:40) does not accept;
#   * no POC(0, 0) when the model has no Nonnegatives rows -- moi.jl:215;
#   * ConstraintPrimal / ConstraintDual without scalecoef, which moi.jl:262,269
#     call but nothing defines (it is the identity for these cones: ECOS.jl
#     scales only PSD cones);
#   * the dual of a Zeros constraint is y, not z -- moi.jl:265 reads z for
#     every constraint;
#   * TerminationStatus / PrimalStatus / BarrierIterations getters (moi.jl has
#     none: the reference returns no status, solver.jl:152).
# `optimize_batched!(opts)` solves many models in one device launch per
# structure class (the batched path the HIP kernels are built for).
#
# The arithmetic and packing mirror socp.jl_amd/socp_amd/moi.py, which the
# repository's tests exercise (tests/test_moi.py); this file is not executed
# here (no Julia in the image).

const HIP_STATUS = Dict(0 => MOI.OPTIMAL, 1 => MOI.ITERATION_LIMIT, 2 => MOI.NUMERICAL_ERROR,
                        3 => MOI.NUMERICAL_ERROR, 4 => MOI.NUMERICAL_ERROR)

mutable struct HipOptimizer <: MOI.AbstractOptimizer
    inner::Optimizer      # the reference adapter: cone bookkeeping + loaded data
    iters::Int32
    status::Int32         # -1: optimize! not called since the last copy_to
    function HipOptimizer(; kwargs...)
        new(Optimizer(; kwargs...), Int32(0), Int32(-1))
    end
end

# ---- model loading: forwarded to the wrapped reference Optimizer
MOI.get(::HipOptimizer, ::MOI.SolverName) = "SOCP.jl (HIP dense path)"
MOI.supports(::HipOptimizer, ::MOI.Silent) = true
MOI.is_empty(o::HipOptimizer) = MOI.is_empty(o.inner)
function MOI.empty!(o::HipOptimizer)
    MOI.empty!(o.inner)
    o.status = Int32(-1)
    o.iters = Int32(0)
end
MOI.supports(o::HipOptimizer, a::Union{MOI.ObjectiveSense, MOI.ObjectiveFunction{MOI.ScalarAffineFunction{Float64}}}) =
    MOI.supports(o.inner, a)
MOI.supports_constraint(o::HipOptimizer, F::Type{<:MOI.AbstractFunction}, S::Type{<:MOI.AbstractSet}) =
    MOI.supports_constraint(o.inner, F, S)
function MOI.copy_to(dest::HipOptimizer, src::MOI.ModelLike; kws...)
    dest.status = Int32(-1)
    return MOI.copy_to(dest.inner, src; kws...)   # moi.jl:95-97 (automatic_copy_to on the inner)
end

# ---- solve
function _hip_problem(o::Optimizer)
    cone = o.cone
    d = o.data
    A = Matrix(sparse(d.IA, d.JA, d.VA, cone.f, d.n))
    G = Matrix(sparse(d.IG, d.JG, d.VG, d.m, d.n))
    cones = Cone[]
    cone.l > 0 && push!(cones, POC(0, cone.l))
    offs = cone.l
    for q in cone.qa
        push!(cones, SOC(offs, q))
        offs += q
    end
    return Problem(d.c, A, d.b, G, d.h, Tuple(cones))
end

_opt(o::Optimizer, key, default) = get(Dict(o.options), key, default)

function optimize_batched!(opts::AbstractVector{HipOptimizer})
    todo = [o for o in opts if o.inner.data !== nothing]
    groups = Dict{Any, Vector{HipOptimizer}}()
    for o in todo
        i = o.inner
        key = (i.data.n, i.cone.f, i.cone.l, Tuple(i.cone.qa), _opt(i, :maxit, 40), _opt(i, :tol, 1e-5))
        push!(get!(groups, key, HipOptimizer[]), o)
    end
    for (key, group) in groups
        probs = [_hip_problem(o.inner) for o in group]
        states, iters, status = solve_socp_batched(probs; maxit=key[5], tol=key[6])
        for (o, st, it, ss) in zip(group, states, iters, status)
            o.inner.sol = st
            o.iters = it
            o.status = ss
            o.inner.data = nothing   # optimize! consumes the copied model (the state moi.jl:201-204 tests for)
        end
    end
    return nothing
end

MOI.optimize!(o::HipOptimizer) = optimize_batched!([o])

# ---- results
MOI.get(o::HipOptimizer, ::MOI.TerminationStatus) =
    o.status < 0 ? MOI.OPTIMIZE_NOT_CALLED : HIP_STATUS[o.status]
MOI.get(o::HipOptimizer, ::MOI.BarrierIterations) = Int(o.iters)
MOI.get(o::HipOptimizer, ::MOI.PrimalStatus) =
    MOI.get(o, MOI.TerminationStatus()) == MOI.OPTIMAL ? MOI.FEASIBLE_POINT : MOI.UNKNOWN_RESULT_STATUS
MOI.get(o::HipOptimizer, ::MOI.ResultCount) = o.status < 0 ? 0 : 1
MOI.get(o::HipOptimizer, a::MOI.VariablePrimal, vi::VI) = o.inner.sol.x[vi.value]    # moi.jl:241-243
MOI.get(o::HipOptimizer, a::MOI.VariablePrimal, vi::Vector{VI}) = MOI.get.(o, Ref(a), vi)
# Zeros / EqualTo primals come from the set constants (moi.jl:250-257, which need no scalecoef)
MOI.get(o::HipOptimizer, a::MOI.ConstraintPrimal, ci::CI{<:MOI.AbstractFunction, MOI.Zeros}) = MOI.get(o.inner, a, ci)
MOI.get(o::HipOptimizer, a::MOI.ConstraintPrimal, ci::CI{<:MOI.AbstractFunction, <:MOI.EqualTo}) = MOI.get(o.inner, a, ci)
function MOI.get(o::HipOptimizer, ::MOI.ConstraintPrimal, ci::CI{<:MOI.AbstractFunction, S}) where S <: MOI.AbstractSet
    i = o.inner
    offset = constroffset(i, ci)
    rows = constrrows(i, ci)
    _unshift(i, offset, reorderval(i.sol.s[offset .+ rows], S), ci)   # moi.jl:259-263 without scalecoef
end
_hip_dual(o::Optimizer, ::CI{<:MOI.AbstractFunction, MOI.Zeros}) = o.sol.y   # equality rows: y (moi.jl:265 reads z)
_hip_dual(o::Optimizer, ::CI) = o.sol.z
function MOI.get(o::HipOptimizer, ::MOI.ConstraintDual, ci::CI{<:MOI.AbstractFunction, S}) where S <: MOI.AbstractSet
    i = o.inner
    offset = constroffset(i, ci)
    rows = constrrows(i, ci)
    reorderval(_hip_dual(i, ci)[offset .+ rows], S)   # moi.jl:266-270 without scalecoef
end
