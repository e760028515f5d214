# SocpHipMOI.jl — routes the reference's MathOptInterface adapter (src/moi.jl)
# to the HIP dense path, with the fixes that keep moi.jl from running as written
# (SURVEY.md §8(f) row 2).  Include inside module Socp after moi.jl and
# SocpHip.jl:
#     include(joinpath(SOCP_AMD_DIR, "julia", "SocpHipMOI.jl"))
#
# Fixes (each cites the reference line it replaces):
#   * optimize! builds SolverState(prob, HipDenseSolver(prob)) — moi.jl:220
#     passes a SparseSolver where a SolverState is expected;
#   * no POC(0,0) when the model has no Nonnegatives rows — moi.jl:212;
#   * cones passed as a Tuple (Problem's type parameter C) — moi.jl:212-217
#     builds a Vector{Cone};
#   * scalecoef (undefined, moi.jl:251,257) is the identity (PSD-only in ECOS.jl);
#   * the dual of a Zeros constraint is y, not z — moi.jl:254;
#   * TerminationStatus / ObjectiveValue / BarrierIterations getters.
# `optimize_batched!(opts)` solves many models in one device launch per
# structure class (the batched path the HIP kernels are built for).
#
# The arithmetic and packing mirror socp.jl_amd/socp_amd/moi.py, which the
# repository's tests exercise (tests/test_moi.py); this file is not executed
# here (no Julia in the image).

const HIP_STATUS = Dict(0 => MOI.OPTIMAL, 1 => MOI.ITERATION_LIMIT, 2 => MOI.NUMERICAL_ERROR,
                        3 => MOI.NUMERICAL_ERROR, 4 => MOI.NUMERICAL_ERROR)

mutable struct HipResult
    iters::Int32
    status::Int32
end
const _hip_results = IdDict{Optimizer, HipResult}()

scalecoef(rows, coef, minus, ::Type) = coef

function _hip_problem(instance::Optimizer)
    cone = instance.cone
    d = instance.data
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

_opt(instance, key, default) = get(Dict(instance.options), key, default)

function optimize_batched!(instances::AbstractVector{Optimizer})
    todo = [o for o in instances if o.data !== nothing]
    groups = Dict{Any, Vector{Optimizer}}()
    for o in todo
        key = (o.data.n, o.cone.f, o.cone.l, Tuple(o.cone.qa), _opt(o, :maxit, 40), _opt(o, :tol, 1e-5))
        push!(get!(groups, key, Optimizer[]), o)
    end
    for (key, opts) in groups
        probs = [_hip_problem(o) for o in opts]
        states, iters, status = solve_socp_batched(probs; maxit=key[5], tol=key[6])
        for (o, st, it, ss) in zip(opts, states, iters, status)
            o.sol = st
            _hip_results[o] = HipResult(it, ss)
            o.data = nothing    # as moi.jl:204-207: optimize! consumes the copied model
        end
    end
    return nothing
end

function MOI.optimize!(instance::Optimizer)
    instance.data === nothing && return
    optimize_batched!([instance])
end

MOI.get(instance::Optimizer, ::MOI.TerminationStatus) =
    haskey(_hip_results, instance) ? HIP_STATUS[_hip_results[instance].status] : MOI.OPTIMIZE_NOT_CALLED
MOI.get(instance::Optimizer, ::MOI.BarrierIterations) = Int(_hip_results[instance].iters)
MOI.get(instance::Optimizer, ::MOI.PrimalStatus) =
    MOI.get(instance, MOI.TerminationStatus()) == MOI.OPTIMAL ? MOI.FEASIBLE_POINT : MOI.UNKNOWN_RESULT_STATUS

_dual(instance, ci::CI{<:MOI.AbstractFunction, MOI.Zeros}) = instance.sol.y
function MOI.get(instance::Optimizer, ::MOI.ConstraintDual, ci::CI{<:MOI.AbstractFunction, MOI.Zeros})
    offset = constroffset(instance, ci)
    rows = constrrows(instance, ci)
    instance.sol.y[offset .+ rows]
end
