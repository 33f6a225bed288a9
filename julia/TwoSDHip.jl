# TwoSDHip.jl -- Julia binding of libtwosd_hip.so for the reference's TwoSD module.
#
# NOT EXECUTED in this repository: the image has no Julia toolchain (no `julia` binary, no
# network to install it).  tests/julia_mirror.py restates this file 1:1 in Python ctypes (same
# entry points, same argument order, 1-based template / position arrays, same call sequence per
# sd_iteration!) and tests/test_gpu_julia_mirror.py drives that mirror on the GPU against an
# oracle replay of algorithm.jl:39-115.
#
# Drop-in for the reference driver (test/instance_test/sd_single_cut_test.jl):
#
#     cell = TwoSD.sdCell(sp1); TwoSD.bind_epigraph!(cell, TwoSD.sdEpigraph(sp2, 1.0, lb))
#     ... set_optimizer(cell.master, ...) as before ...
#     cell = TwoSDHip.HipCell(cell, sto)                    # <- the one added line
#     TwoSD.sd_iteration!(cell, [rand(sto)]; quad_scalar_schedule=...)     # unchanged
#     cell.improvement_info, cell.x_incumbent, cell.ext, length(cell.dual_vertices)   # unchanged
#
# `sdCell` types its fields concretely (epi::Vector{sdEpigraph}, dual_vertices::sdDualVertexSet,
# cell.jl:18,26), so the accelerated state cannot live inside it.  HipCell wraps the reference
# cell, forwards every field to it (getproperty / setproperty!) except `dual_vertices`, which is
# the device set, and has its own `TwoSD.sd_iteration!` method: algorithm.jl:39-115 line for line,
# with the scenario solves, the dual pushes and the cuts on the GPU and the JuMP master, cut
# removal, sync_cuts!, incumbent selection and the prox schedule left to the reference's code on
# the reference's objects.  That method is the only method this module adds to a TwoSD function;
# everything else is a TwoSDHip function.
module TwoSDHip
using ..TwoSD, SparseArrays, JuMP, LinearAlgebra
const MOI = JuMP.MOI
const LIB = joinpath(@__DIR__, "..", "sqlp_amd", "libtwosd_hip.so")

check(rc) = rc == 0 || error(unsafe_string(ccall((:twosd_last_error, LIB), Cstring, ())))

# ---------------------------------------------------------------------------------------------
# Device context: stage-2 template + random-element layout + warm-start basis + vertex set
mutable struct HipContext                     # one per cell per GPU; finalizer frees device memory
    h::Ptr{Cvoid}
    nrow::Int; n1::Int; n2::Int
    positions::Vector{TwoSD.spSmpsPosition}
    has_basis::Bool
end

row_sense(c) = c isa ConstraintRef{<:Any,<:MOI.ConstraintIndex{<:Any,MOI.GreaterThan{Float64}}} ? UInt8('G') :
               c isa ConstraintRef{<:Any,<:MOI.ConstraintIndex{<:Any,MOI.LessThan{Float64}}} ? UInt8('L') : UInt8('E')

# extract_coefficients (subprob.jl:15-69) handed to twosd_set_template as Julia arrays (1-based)
function HipContext(sp2::TwoSD.spStageProblem, sto::TwoSD.spStoType; device::Int=0)
    ref = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:twosd_create, LIB), Cint, (Cint, Ref{Ptr{Cvoid}}), device, ref))
    coef = TwoSD.extract_coefficients(sp2)
    T = SparseMatrixCSC(coef.transfer); W = SparseMatrixCSC(coef.recourse)
    q = Float64[coefficient(objective_function(sp2.model), v) for v in sp2.current_stage_vars]
    sense = UInt8[row_sense(c) for c in sp2.stage_constraints]
    r = Vector{Float64}(coef.rhs)
    check(ccall((:twosd_set_template, LIB), Cint,
        (Ptr{Cvoid}, Cint, Cint, Cint, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Ptr{Int64}, Ptr{Int64}, Ptr{Float64},
         Ptr{Float64}, Ptr{Float64}, Ptr{UInt8}, Ptr{Float64}, Ptr{Float64}, Cint),
        ref[], size(T, 1), size(T, 2), size(W, 2), T.colptr, T.rowval, T.nzval, W.colptr, W.rowval, W.nzval,
        q, r, sense, C_NULL, C_NULL, 1))                        # index_base = 1: Julia arrays as-is
    pos = collect(keys(sto.indep))
    rows = Cint[coef.row_lookup[p.row_name] for p in pos]       # KeyError as subprob.jl:112,116
    cols = Cint[p.col_name in ("RHS", "rhs") ? -1 : coef.col_lookup[p.col_name] for p in pos]
    check(ccall((:twosd_set_random_positions, LIB), Cint, (Ptr{Cvoid}, Cint, Ptr{Cint}, Ptr{Cint}, Cint),
                ref[], length(pos), rows, cols, 1))
    ctx = HipContext(ref[], size(T, 1), size(T, 2), size(W, 2), pos, false)
    finalizer(c -> ccall((:twosd_destroy, LIB), Cint, (Ptr{Cvoid},), c.h), ctx)
    return ctx
end

element_values(ctx::HipContext, ω::TwoSD.spSmpsScenario) = (d = Dict(ω); Float64[d[p] for p in ctx.positions])

# Warm-start basis: the optimal basis of one scenario at x (any cost signs; phase 1 on the host
# when the slack basis is not dual feasible).  The randomness is RHS-only, so it is dual
# feasible for every scenario and every x (set once per template).
function compute_basis!(ctx::HipContext, x::Vector{Float64}, ω::TwoSD.spSmpsScenario)
    check(ccall((:twosd_compute_basis, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}),
                ctx.h, x, element_values(ctx, ω)))
    ctx.has_basis = true
end

# solve_problem!(sp, x, ω) -> (obj, y, π) of smps_routines.jl:50-62 on the device
function solve_problem(ctx::HipContext, x::Vector{Float64}, ω::TwoSD.spSmpsScenario)
    obj = Ref(0.0); st = Ref{Cint}(0); y = zeros(ctx.n2); π = zeros(ctx.nrow)
    v = element_values(ctx, ω)
    GC.@preserve v y π check(ccall((:twosd_solve_values, LIB), Cint,
        (Ptr{Cvoid}, Ptr{Float64}, Cint, Ptr{Float64}, Ref{Float64}, Ptr{Float64}, Ptr{Float64}, Ref{Cint}),
        ctx.h, x, 1, v, obj, π, y, st))
    return obj[], y, π
end

# ---------------------------------------------------------------------------------------------
# Device side of one sdEpigraph: its scenario deltas and weights (epigraph.jl:17-61)
struct HipEpigraph; ctx::HipContext; index::Cint; end
function HipEpigraph(ctx::HipContext)
    e = Ref{Cint}(0); check(ccall((:twosd_epigraph_create, LIB), Cint, (Ptr{Cvoid}, Ref{Cint}), ctx.h, e))
    HipEpigraph(ctx, e[])
end
# add_scenario!(epi, ω, w) (epigraph.jl:81-96), device copy
add_scenario!(epi::HipEpigraph, ω::TwoSD.spSmpsScenario, weight::Float64=1.0) =
    check(ccall((:twosd_add_scenarios, LIB), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{Float64}, Ref{Float64}),
                epi.ctx.h, epi.index, 1, element_values(epi.ctx, ω), weight))
function num_scenarios(epi::HipEpigraph)
    n = Ref{Cint}(0)
    check(ccall((:twosd_epigraph_info, LIB), Cint, (Ptr{Cvoid}, Cint, Ref{Cint}, Ptr{Float64}),
                epi.ctx.h, epi.index, n, C_NULL))
    return Int(n[])
end

# solve_problem! + push!(cell.dual_vertices, π) for scenarios [first, first + count) (0-based)
# of epi at x (algorithm.jl:49-50, 53-54), without a host round trip of π
function solve_push!(epi::HipEpigraph, x::Vector{Float64}, first::Integer, count::Integer)
    n = Ref{Cint}(0)
    check(ccall((:twosd_solve_push, LIB), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Float64}, Cint, Cint, Ptr{Float64}, Ptr{Cint}, Ref{Cint}),
        epi.ctx.h, epi.index, x, first, count, C_NULL, C_NULL, n))
    return Int(n[])
end

# incumbent objective of the last solve_push! / solve batch: (sum_s w_s obj_s, sum_s w_s) over its
# scenarios (fixed-order device reduction); across ranks the caller sums both before dividing
function last_objective(ctx::HipContext)
    a = Ref(0.0); b = Ref(0.0)
    check(ccall((:twosd_last_objective, LIB), Cint, (Ptr{Cvoid}, Ref{Float64}, Ref{Float64}), ctx.h, a, b))
    return a[], b[]
end

# build_sasa_cut(epi, x, V) -> sdCut (epigraph.jl:125-146; argmax_procedure subprob.jl:141-169).
# tie_rel = 0 is the reference's strict '>' (first maximum in insertion order).
function build_sasa_cut(epi::HipEpigraph, x::Vector{Float64}; tie_rel::Float64=0.0)
    α = Ref(0.0); wm = Ref(0.0); β = zeros(epi.ctx.n1)
    check(ccall((:twosd_build_cut, LIB), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Float64}, Cdouble, Ref{Float64}, Ptr{Float64}, Ref{Float64}, Ptr{Float64}, Ptr{Cint}),
        epi.ctx.h, epi.index, x, tie_rel, α, β, wm, C_NULL, C_NULL))
    return TwoSD.sdCut(α[], β, wm[])
end

# The cell's dual vertex set lives on the device (dual_set.jl:69-127); push!/length as the reference
struct HipDualVertexSet; ctx::HipContext; end
function Base.push!(V::HipDualVertexSet, π::Vector{Float64})
    n = Ref{Cint}(0)
    check(ccall((:twosd_dvs_push, LIB), Cint, (Ptr{Cvoid}, Cint, Ptr{Float64}, Ptr{Cint}, Ref{Cint}),
                V.ctx.h, 1, π, C_NULL, n))
    return V
end
Base.length(V::HipDualVertexSet) = (n = Ref{Cint}(0);
    check(ccall((:twosd_dvs_size, LIB), Cint, (Ptr{Cvoid}, Ref{Cint}), V.ctx.h, n)); Int(n[]))
# ranks compare this before a cut all-reduce (identical ordered vertex sets)
fingerprint(V::HipDualVertexSet) = (d = Ref{UInt64}(0);
    check(ccall((:twosd_dvs_fingerprint, LIB), Cint, (Ptr{Cvoid}, Ref{UInt64}), V.ctx.h, d)); d[])

# ---------------------------------------------------------------------------------------------
# The accelerated cell
mutable struct HipCell
    cell::TwoSD.sdCell                      # the reference cell: JuMP master, epi (cuts, weights), x's
    ctx::HipContext
    hepi::Vector{HipEpigraph}               # hepi[i] = device side of cell.epi[i]
    dual_vertices::HipDualVertexSet         # replaces cell.dual_vertices (cell.jl:26)
    tie_rel::Float64
end

# Wrap a cell whose epigraphs are bound (cell.jl:99-116).  All epigraphs share one stage-2
# template (every reference driver binds copies of one sp2); the context is built from epi 1's.
function HipCell(cell::TwoSD.sdCell, sto::TwoSD.spStoType; device::Int=0, tie_rel::Float64=0.0)
    isempty(cell.epi) && error("HipCell: bind the epigraphs first (bind_epigraph!)")
    ctx = HipContext(cell.epi[1].prob, sto; device=device)
    c1 = cell.epi[1].subproblem_coef
    for epi in cell.epi[2:end]
        c = epi.subproblem_coef
        (c.rhs == c1.rhs && c.transfer == c1.transfer && c.recourse == c1.recourse) ||
            error("HipCell: epigraphs with different stage-2 templates need one HipCell each")
    end
    hepi = HipEpigraph[HipEpigraph(ctx) for _ in cell.epi]
    for (h, epi) in zip(hepi, cell.epi)     # scenarios added before wrapping (algorithm.jl:46)
        for (ω, w) in zip(epi.scenario_list, epi.scenario_weight)
            add_scenario!(h, ω, w)
        end
    end
    return HipCell(cell, ctx, hepi, HipDualVertexSet(ctx), tie_rel)
end

const OWN = (:cell, :ctx, :hepi, :dual_vertices, :tie_rel)
Base.getproperty(hc::HipCell, s::Symbol) = s in OWN ? getfield(hc, s) : getproperty(getfield(hc, :cell), s)
Base.setproperty!(hc::HipCell, s::Symbol, v) =
    s in OWN ? setfield!(hc, s, v) : setproperty!(getfield(hc, :cell), s, v)

function Base.show(io::IO, hc::HipCell)                           # cell.jl:76-94 with the device set
    cell = hc.cell
    println(io, "HipCell")
    con_cnt = num_constraints(cell.master; count_variable_in_set_constraints = false)
    println(io, "Master con_cnt=$con_cnt var_cnt=$(num_variables(cell.master)) dual_cnt=$(length(hc.dual_vertices))")
    inc_cut_cnt = length([con for con in cell.epicon_incumbent_ref if con !== nothing])
    println(io, "Master Cuts inc=$inc_cut_cnt reg=$([length(cons) for cons in cell.epicon_ref])")
    println(io, "Epigraph cnt=$(length(cell.epi))")
    for epi in cell.epi
        println(io, epi)
    end
end

# sd_iteration!(cell, scenario_list; update_incumbent_cut, quad_scalar_schedule), algorithm.jl:39-115
function TwoSD.sd_iteration!(hc::HipCell, scenario_list::Vector{TwoSD.spSmpsScenario};
        update_incumbent_cut::Bool=true, quad_scalar_schedule::Function=TwoSD.ConstantQuadScalarSchedule(0.1))
    cell = hc.cell
    @assert(length(scenario_list) == length(cell.epivar_ref))                         # :42
    if !hc.ctx.has_basis
        compute_basis!(hc.ctx, cell.x_candidate, scenario_list[1])
    end

    # Solve the subproblem (:45-55)
    for i in eachindex(scenario_list)
        TwoSD.add_scenario!(cell.epi[i], scenario_list[i], 1.0)     # host record: weights, total weight
        add_scenario!(hc.hepi[i], scenario_list[i], 1.0)            # device deltas
        s = num_scenarios(hc.hepi[i]) - 1
        solve_push!(hc.hepi[i], cell.x_candidate, s, 1)             # solve at candidate + push!
        solve_push!(hc.hepi[i], cell.x_incumbent, s, 1)             # solve at incumbent + push!
    end

    # Remove cuts with non-zero multiplier (:57-72)
    if termination_status(cell.master) in [OPTIMAL, LOCALLY_SOLVED]
        for i in eachindex(cell.epicon_ref)
            delete_index = Int[]
            for j in eachindex(cell.epicon_ref[i])
                if abs(dual(cell.epicon_ref[i][j])) < TwoSD.CUT_REMOVE_TOLERANCE
                    push!(delete_index, j)
                end
            end
            deleteat!(cell.epi[i].cuts, delete_index)
        end
    end

    epi_info_last = TwoSD.sdEpigraphInfo[TwoSD.sdEpigraphInfo(epi) for epi in cell.epi]   # :76

    # Generate cuts (:79-85)
    for (i, epi) in enumerate(cell.epi)
        push!(epi.cuts, build_sasa_cut(hc.hepi[i], cell.x_candidate; tie_rel=hc.tie_rel))
        if update_incumbent_cut
            epi.incumbent_cut = build_sasa_cut(hc.hepi[i], cell.x_incumbent; tie_rel=hc.tie_rel)
        end
    end

    cell.improvement_info = TwoSD.check_improvement(epi_info_last, cell.epi,
        cell.x_candidate, cell.x_incumbent, cell.x_ref, cell.objf_original)           # :89-90
    rho = quad_scalar_schedule(cell)                                                  # :94
    if cell.improvement_info.is_improved
        cell.x_incumbent .= cell.x_candidate
    end
    TwoSD.add_regularization!(cell, cell.x_incumbent, rho)                           # :101-102
    TwoSD.sync_cuts!(cell)
    try
        optimize!(cell.master)
        @assert(termination_status(cell.master) in [OPTIMAL, LOCALLY_SOLVED])
    catch
        write_to_file(cell.master, "error_model.mof.json")
        rethrow()
    end
    cell.x_candidate .= value.(cell.x_ref)                                            # :112
    return
end

# ---------------------------------------------------------------------------------------------
# Batched entry points (no reference counterpart: the reference drivers are sequential)

# rand(sto) on the device: N scenarios straight into an epigraph        smps_sto.jl:117-149
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

# evaluate(sp1, sp2, sto, x; N) with device-drawn scenarios             smps_routines.jl:67-82
# (needs set_distributions!; s1_cost = c'x of the root stage)
function evaluate(ctx::HipContext, s1_cost::Float64, x::Vector{Float64}, N::Int, seed::UInt64)
    s2 = Ref(0.0)
    check(ccall((:twosd_evaluate_sampled, LIB), Cint, (Ptr{Cvoid}, Ptr{Float64}, Int64, Int64, Int64, UInt64, Ref{Float64}),
                ctx.h, x, N, 0, N, seed, s2))
    return s1_cost + s2[]
end

# warm-start basis pool (fewer pivots, same optima): built once, refreshed at a new x
pool_build!(ctx::HipContext, epi::HipEpigraph, x::Vector{Float64}, count::Integer, max_pool::Integer) =
    (n = Ref{Cint}(0); check(ccall((:twosd_pool_build, LIB), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Float64}, Cint, Cint, Cint, Ref{Cint}), ctx.h, epi.index, x, 0, count, max_pool, n)); n[])
pool_build_candidates!(ctx::HipContext, epi::HipEpigraph, x::Vector{Float64}, count::Integer, level1::Integer,
                       ncand::Integer) =
    check(ccall((:twosd_pool_build_candidates, LIB), Cint, (Ptr{Cvoid}, Cint, Ptr{Float64}, Cint, Cint, Cint, Cint),
                ctx.h, epi.index, x, 0, count, level1, ncand))
pool_refresh!(ctx::HipContext, epi::HipEpigraph, x::Vector{Float64}, count::Integer, max_pool::Integer) =
    (n = Ref{Cint}(0); check(ccall((:twosd_pool_refresh, LIB), Cint,
        (Ptr{Cvoid}, Cint, Ptr{Float64}, Cint, Cint, Cint, Ref{Cint}), ctx.h, epi.index, x, 0, count, max_pool, n)); n[])

# multi-GPU split of build_sasa_cut: partial sums into caller-owned DEVICE buffers (e.g.
# ROCArray memory), all-reduce them with RCCL / MPI, then finalize on every rank
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
end # module
