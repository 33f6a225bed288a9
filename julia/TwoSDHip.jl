# TwoSDHip.jl -- Julia binding of libtwosd_hip.so for the reference's TwoSD module.
#
# NOT EXECUTED in this repository: the image has no Julia toolchain (no `julia` binary, no
# network to install it).  Every entry point it binds is exercised through the identical C
# ABI (include/twosd_hip.h) by the Python ctypes host layer (sqlp_amd/twosd.py) that the
# test suite drives, including the 1-based index path used here (index_base = 1;
# tests/test_gpu_parity_paths.py::test_index_base_one_matches_base_zero).
#
# Usage from the reference checkout:  include("TwoSDHip.jl"); using .TwoSDHip
#   ctx = TwoSDHip.HipContext(sp2, sto); TwoSDHip.compute_basis!(ctx, x, scenario)
#   epi = TwoSDHip.HipEpigraph(ctx); V = TwoSDHip.HipDualVertexSet(ctx)
#   TwoSD.add_scenario!(epi, ω); π = TwoSD.solve_problem!(ctx, x, ω)[3]; push!(V, π)
#   cut = TwoSD.build_sasa_cut(epi, x, V)
module TwoSDHip
using ..TwoSD, SparseArrays, JuMP
const LIB = joinpath(@__DIR__, "..", "sqlp_amd", "libtwosd_hip.so")

check(rc) = rc == 0 || error(unsafe_string(ccall((:twosd_last_error, LIB), Cstring, ())))

mutable struct HipContext                     # one per cell per GPU; finalizer frees device memory
    h::Ptr{Cvoid}
    nrow::Int; n1::Int; n2::Int
    positions::Vector{TwoSD.spSmpsPosition}
end
function HipContext(sp2::TwoSD.spStageProblem, sto::TwoSD.spStoType; device::Int=0)
    ref = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:twosd_create, LIB), Cint, (Cint, Ref{Ptr{Cvoid}}), device, ref))
    coef = TwoSD.extract_coefficients(sp2)                  # subprob.jl:15-69
    T = SparseMatrixCSC(coef.transfer); W = SparseMatrixCSC(coef.recourse)
    q = [coefficient(objective_function(sp2.model), v) for v in sp2.current_stage_vars]
    sense = UInt8[c isa ConstraintRef{<:Any,<:MOI.ConstraintIndex{<:Any,MOI.GreaterThan{Float64}}} ? 'G' :
                  c isa ConstraintRef{<:Any,<:MOI.ConstraintIndex{<:Any,MOI.LessThan{Float64}}} ? 'L' : 'E'
                  for c in sp2.stage_constraints]
    r = Vector(coef.rhs)
    check(ccall((:twosd_set_template, LIB), Cint,
        (Ptr{Cvoid}, Cint, Cint, Cint, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Ptr{Int64}, Ptr{Int64}, Ptr{Float64},
         Ptr{Float64}, Ptr{Float64}, Ptr{UInt8}, Ptr{Float64}, Ptr{Float64}, Cint),
        ref[], size(T, 1), size(T, 2), size(W, 2), T.colptr, T.rowval, T.nzval, W.colptr, W.rowval, W.nzval,
        q, r, sense, C_NULL, C_NULL, 1))                        # index_base = 1: Julia arrays as-is
    pos = collect(keys(sto.indep))
    rows = Cint[coef.row_lookup[p.row_name] for p in pos]
    cols = Cint[p.col_name in ("RHS", "rhs") ? -1 : coef.col_lookup[p.col_name] for p in pos]
    check(ccall((:twosd_set_random_positions, LIB), Cint, (Ptr{Cvoid}, Cint, Ptr{Cint}, Ptr{Cint}, Cint),
                ref[], length(pos), rows, cols, 1))
    ctx = HipContext(ref[], size(T, 1), size(T, 2), size(W, 2), pos)
    finalizer(c -> ccall((:twosd_destroy, LIB), Cint, (Ptr{Cvoid},), c.h), ctx)
    return ctx
end

values(ctx, ω::TwoSD.spSmpsScenario) = [Dict(ω)[p] for p in ctx.positions]

# warm-start basis (once per template; any x)
compute_basis!(ctx, x, ω) = check(ccall((:twosd_compute_basis, LIB), Cint,
    (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}), ctx.h, x, values(ctx, ω)))

# solve_problem!(sp, x, ω) -> (obj, y, π)            smps_routines.jl:50-62
function TwoSD.solve_problem!(ctx::HipContext, x::Vector{Float64}, ω::TwoSD.spSmpsScenario)
    obj = Ref(0.0); st = Ref{Cint}(0); y = zeros(ctx.n2); π = zeros(ctx.nrow)
    v = values(ctx, ω)
    GC.@preserve v y π check(ccall((:twosd_solve_values, LIB), Cint,
        (Ptr{Cvoid}, Ptr{Float64}, Cint, Ptr{Float64}, Ref{Float64}, Ptr{Float64}, Ptr{Float64}, Ref{Cint}),
        ctx.h, x, 1, v, obj, π, y, st))
    return obj[], y, π
end

# epigraphs: add_scenario!(epi, ω, w)                 epigraph.jl:81-96
struct HipEpigraph; ctx::HipContext; index::Cint; end
function HipEpigraph(ctx::HipContext)
    e = Ref{Cint}(0); check(ccall((:twosd_epigraph_create, LIB), Cint, (Ptr{Cvoid}, Ref{Cint}), ctx.h, e))
    HipEpigraph(ctx, e[])
end
TwoSD.add_scenario!(epi::HipEpigraph, ω::TwoSD.spSmpsScenario, weight::Float64=1.0) =
    check(ccall((:twosd_add_scenarios, LIB), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{Float64}, Ref{Float64}),
                epi.ctx.h, epi.index, 1, values(epi.ctx, ω), weight))

# rand(sto) on the device: N scenarios straight into the epigraph   smps_sto.jl:117-149
function set_distributions!(ctx::HipContext, sto::TwoSD.spStoType)
    kind = Cint[]; ns = Cint[]; vals = Float64[]; probs = Float64[]; p0 = Float64[]; p1 = Float64[]
    for pos in ctx.positions
        d = sto.indep[pos]
        if d isa TwoSD.spSmpsDiscreteDistribution
            push!(kind, 0); push!(ns, length(d.value)); append!(vals, d.value); append!(probs, d.probability)
            push!(p0, 0.0); push!(p1, 0.0)
        elseif d isa TwoSD.spSmpsNormalDistribution
            push!(kind, 1); push!(ns, 0); push!(p0, d.mean); push!(p1, d.variance)
        else
            push!(kind, 2); push!(ns, 0); push!(p0, d.left); push!(p1, d.right)
        end
    end
    check(ccall((:twosd_set_distributions, LIB), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Cint}, Ptr{Cint}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
        ctx.h, length(kind), kind, ns, vals, probs, p0, p1))
end
add_sampled_scenarios!(epi::HipEpigraph, N::Integer, seed::UInt64; first::UInt64=UInt64(0)) =
    check(ccall((:twosd_add_sampled_scenarios, LIB), Cint, (Ptr{Cvoid}, Cint, Cint, UInt64, UInt64, Ptr{Float64}),
                epi.ctx.h, epi.index, N, seed, first, C_NULL))

# evaluate(sp1, sp2, sto, x; N) with device-drawn scenarios          smps_routines.jl:67-82
function TwoSD.evaluate(ctx::HipContext, s1_cost::Float64, x::Vector{Float64}, N::Int, seed::UInt64)
    s2 = Ref(0.0)
    check(ccall((:twosd_evaluate_sampled, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}, Int64, Int64, Int64, UInt64, Ref{Float64}),
                ctx.h, x, N, 0, N, seed, s2))
    return s1_cost + s2[]
end

# warm-start basis pool: optimal bases of training scenarios (setup; fewer pivots, same optima)
pool_build!(ctx::HipContext, epi::HipEpigraph, x::Vector{Float64}, count::Integer, max_pool::Integer) =
    (n = Ref{Cint}(0); check(ccall((:twosd_pool_build, LIB), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Float64}, Cint, Cint, Cint, Ref{Cint}), ctx.h, epi.index, x, 0, count, max_pool, n)); n[])
# two-level selection over a large pool (setup): level 1 = the `level1` most frequent bases,
# level 2 = `ncand` learned candidates per level-1 pick (bench: 32768 bases at 1M scenarios per GPU, 16384 below; 128 + 160)
pool_build_candidates!(ctx::HipContext, epi::HipEpigraph, x::Vector{Float64}, count::Integer, level1::Integer,
                       ncand::Integer) =
    check(ccall((:twosd_pool_build_candidates, LIB), Cint, (Ptr{Cvoid}, Cint, Ptr{Float64}, Cint, Cint, Cint, Cint),
                ctx.h, epi.index, x, 0, count, level1, ncand))

# per-x pool (timed in the bench): rebuilt from the optimal bases of training scenarios at x
pool_refresh!(ctx::HipContext, epi::HipEpigraph, x::Vector{Float64}, count::Integer, max_pool::Integer) =
    (n = Ref{Cint}(0); check(ccall((:twosd_pool_refresh, LIB), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Float64}, Cint, Cint, Cint, Ref{Cint}), ctx.h, epi.index, x, 0, count, max_pool, n)); n[])

# push!(::sdDualVertexSet, π)                         dual_set.jl:84-94 (the set lives on the GPU)
struct HipDualVertexSet; ctx::HipContext; end
function Base.push!(V::HipDualVertexSet, π::Vector{Float64})
    n = Ref{Cint}(0)
    check(ccall((:twosd_dvs_push, LIB), Cint, (Ptr{Cvoid}, Cint, Ptr{Float64}, Ptr{Cint}, Ref{Cint}),
                V.ctx.h, 1, π, C_NULL, n))
    return V
end
Base.length(V::HipDualVertexSet) = (n = Ref{Cint}(0);
    check(ccall((:twosd_dvs_size, LIB), Cint, (Ptr{Cvoid}, Ref{Cint}), V.ctx.h, n)); Int(n[]))

# build_sasa_cut(epi, x, V) -> sdCut                 epigraph.jl:125-146 (argmax: subprob.jl:141-169)
function TwoSD.build_sasa_cut(epi::HipEpigraph, x::Vector{Float64}, V::HipDualVertexSet; tie_rel=1e-12)
    α = Ref(0.0); wm = Ref(0.0); β = zeros(epi.ctx.n1)
    check(ccall((:twosd_build_cut, LIB), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Float64}, Cdouble, Ref{Float64}, Ptr{Float64}, Ref{Float64}, Ptr{Float64}, Ptr{Cint}),
        epi.ctx.h, epi.index, x, tie_rel, α, β, wm, C_NULL, C_NULL))
    return TwoSD.sdCut(α[], β, wm[])
end

# batched sd_iteration! segment on the device (algorithm.jl:45-55): solve scenarios
# [first, first + count) of epi at x and push their duals into V without a host round trip
function solve_push!(epi::HipEpigraph, x::Vector{Float64}, first::Integer, count::Integer)
    obj = zeros(count); st = zeros(Cint, count); n = Ref{Cint}(0)
    check(ccall((:twosd_solve_push, LIB), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Float64}, Cint, Cint, Ptr{Float64}, Ptr{Cint}, Ref{Cint}),
        epi.ctx.h, epi.index, x, first, count, obj, st, n))
    return obj, Int(n[])
end

# multi-GPU split of build_sasa_cut: partial sums into caller-owned DEVICE buffers (e.g.
# CuArray / ROCArray memory), all-reduce them with RCCL / MPI, then finalize on every rank
function cut_partial_len(ctx::HipContext)
    a = Ref{Int64}(0); b = Ref{Int64}(0)
    check(ccall((:twosd_cut_partial_len, LIB), Cint, (Ptr{Cvoid}, Ref{Int64}, Ref{Int64}), ctx.h, a, b))
    return a[], b[]
end
cut_partial!(epi::HipEpigraph, x, tie_rel, total_weight, d_hist::Ptr{UInt64}, d_sums::Ptr{Float64}) =
    check(ccall((:twosd_cut_partial, LIB), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Float64}, Cdouble, Cdouble, Ptr{UInt64}, Ptr{Float64}, Ptr{Float64}, Ptr{Cint}),
        epi.ctx.h, epi.index, x, tie_rel, total_weight, d_hist, d_sums, C_NULL, C_NULL))
function cut_finalize(ctx::HipContext, x, d_hist::Ptr{UInt64}, d_sums::Ptr{Float64})
    α = Ref(0.0); β = zeros(ctx.n1)
    check(ccall((:twosd_cut_finalize, LIB), Cint,
        (Ptr{Cvoid}, Ptr{Float64}, Ptr{UInt64}, Ptr{Float64}, Ref{Float64}, Ptr{Float64}),
        ctx.h, x, d_hist, d_sums, α, β))
    return α[], β
end
# ranks compare this before the all-reduce (identical ordered vertex sets)
fingerprint(V::HipDualVertexSet) = (d = Ref{UInt64}(0);
    check(ccall((:twosd_dvs_fingerprint, LIB), Cint, (Ptr{Cvoid}, Ref{UInt64}), V.ctx.h, d)); d[])
end # module
