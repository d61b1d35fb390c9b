# MadIPM package extension for AMD GPUs (MI355X, gfx950) over libmadipm_hip.so.
#
# Mirrors the reference's ext/MadIPMCUDAExt/MadIPMCUDAExt.jl + cuda_wrapper.jl: the same methods,
# specialised on ROCArray / AMDGPU.rocSPARSE types, with every kernel a C-ABI entry point of the
# library (include/madipm_hip.h) instead of a KernelAbstractions/cuSPARSE kernel, plus the
# linear-solver plugin `HIPLDLSolver` (the cuDSS counterpart: MadNLP.AbstractLinearSolver) and
# `madipm_hip`, the whole-solver route (native MPC driver).
#
# Wiring (in MadIPM's Project.toml, next to the CUDA extension):
#   [weakdeps]    AMDGPU = "21141c5a-9bdb-4563-92ae-f87d6854732e"
#   [extensions]  MadIPMHIPExt = "AMDGPU"
# Use:
#   qp_gpu = convert(QuadraticModel{Float64, ROCVector{Float64}}, qp)
#   madipm(qp_gpu; linear_solver = MadIPMHIPExt.HIPLDLSolver)        # reference MPC loop, our LDL^T
#   MadIPMHIPExt.madipm_hip(qp)                                       # everything on the GPU
#
# Not executed in this repository (no Julia toolchain in the image); the Python mirror
# (madipm.jl_amd/madipm_amd) binds the same symbols and is what the tests run.
module MadIPMHIPExt

using LinearAlgebra
using SparseArrays
using NLPModels
using QuadraticModels
using AMDGPU
using AMDGPU.rocSPARSE
import QuadraticModels: SparseMatrixCOO
import MadNLP
import MadIPM

include("hip_wrapper.jl")

# ------------------------------------------------------------ QP evaluators (MadIPMCUDAExt.jl:15-87)
function fill_structure!(A::ROCSparseMatrixCSR, rows, cols)
    @assert length(cols) == length(rows)
    length(cols) == 0 && return
    rp0 = zero_based(A.rowPtr)
    ci0 = zero_based(A.colVal)
    r0 = ROCVector{Int32}(undef, length(rows))
    c0 = ROCVector{Int32}(undef, length(cols))
    GC.@preserve rp0 ci0 r0 c0 check(ccall((:madipm_csr_fill_structure, libmadipm), Cint,
        (Int32, Ptr{Int32}, Ptr{Int32}, Ptr{Int32}, Ptr{Int32}, Ptr{Cvoid}),
        size(A, 1), pointer(rp0), pointer(ci0), pointer(r0), pointer(c0), hipstream()), "madipm_csr_fill_structure")
    rows .= r0 .+ one(eltype(rows))
    cols .= c0 .+ one(eltype(cols))
    return
end

const OBJ_WORK = Ref{Any}(nothing)

function NLPModels.obj(qp::QuadraticModel{T, S, M1}, x::AbstractVector) where {T, S, M1 <: MadIPMOperator}
    NLPModels.increment!(qp, :neval_obj)
    work = OBJ_WORK[]
    (work === nothing) && (work = OBJ_WORK[] = ROCVector{Float64}(undef, 513))
    obj = Ref{Float64}(0.0)
    GC.@preserve qp x work check(ccall((:madipm_qp_obj, libmadipm), Cint,
        (Ptr{Cvoid}, Ptr{Float64}, Float64, Ptr{Float64}, Ptr{Float64}, Int32, Ptr{Float64}, Ref{Float64}, Ptr{Cvoid}),
        qp.data.H.handle, pointer(qp.data.c), qp.data.c0, pointer(x), pointer(qp.data.v), length(x), pointer(work),
        obj, hipstream()), "madipm_qp_obj")
    return obj[]                                    # c0 + c'x + (Hx)'x / 2
end

function NLPModels.grad!(qp::QuadraticModel{T, S, M1}, x::AbstractVector, g::AbstractVector) where {T, S, M1 <: MadIPMOperator}
    NLPModels.increment!(qp, :neval_grad)
    GC.@preserve qp x g check(ccall((:madipm_qp_grad, libmadipm), Cint,
        (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int32, Ptr{Cvoid}),
        qp.data.H.handle, pointer(qp.data.c), pointer(x), pointer(g), length(x), hipstream()), "madipm_qp_grad")
    return g                                         # H x + c
end

function NLPModels.hess_structure!(qp::QuadraticModel{T, S, M1}, rows::AbstractVector{<:Integer},
                                   cols::AbstractVector{<:Integer}) where {T, S, M1 <: MadIPMOperator}
    fill_structure!(qp.data.H.A, rows, cols)
    return rows, cols
end

function NLPModels.hess_coord!(qp::QuadraticModel{T, S, M1}, x::AbstractVector{T}, vals::AbstractVector{T};
                               obj_weight::Real = one(eltype(x))) where {T, S, M1 <: MadIPMOperator}
    NLPModels.increment!(qp, :neval_hess)
    vals .= obj_weight .* qp.data.H.A.nzVal
    return vals
end

function NLPModels.jac_lin_coord!(qp::QuadraticModel{T, S, M1, M2}, x::AbstractVector,
                                  vals::AbstractVector) where {T, S, M1, M2 <: MadIPMOperator}
    @lencheck qp.meta.nvar x
    @lencheck qp.meta.lin_nnzj vals
    NLPModels.increment!(qp, :neval_jac_lin)
    vals .= qp.data.A.A.nzVal
    return vals
end

function NLPModels.jac_lin_structure!(qp::QuadraticModel{T, S, M1, M2}, rows::AbstractVector{<:Integer},
                                      cols::AbstractVector{<:Integer}) where {T, S, M1, M2 <: MadIPMOperator}
    @lencheck qp.meta.lin_nnzj rows cols
    fill_structure!(qp.data.A.A, rows, cols)
    return rows, cols
end

# ------------------------------------------------------------ device sparse matrices (MadIPMCUDAExt.jl:89-116)
rocSPARSE.ROCSparseMatrixCOO(A::SparseMatrixCOO{Tv, Ti}) where {Tv, Ti} =
    rocSPARSE.ROCSparseMatrixCOO{Tv, Ti}(ROCVector(A.rows), ROCVector(A.cols), ROCVector(A.vals), size(A), nnz(A))

function rocSPARSE.ROCSparseMatrixCSR(A::SparseMatrixCOO{Tv, Ti}) where {Tv, Ti}
    m, n = size(A)
    Ap, Ai, Ax = MadIPM.coo_to_csr(m, n, ROCVector{Int32}(A.rows), ROCVector{Int32}(A.cols), ROCVector(A.vals))
    return rocSPARSE.ROCSparseMatrixCSR{Tv, Ti}(ROCVector{Ti}(Ap), ROCVector{Ti}(Ai), ROCVector(Ax), size(A))
end

# ------------------------------------------------------------ QuadraticModel on the GPU (MadIPMCUDAExt.jl:118-137)
function Base.convert(::Type{QuadraticModel{T, S}}, qp::QuadraticModel{T}) where {T, S<:ROCArray}
    H = MadIPMOperator(ROCSparseMatrixCSR(qp.data.H), symmetric=true)
    A = MadIPMOperator(ROCSparseMatrixCSR(qp.data.A), symmetric=false)
    return QuadraticModel(S(qp.data.c), H; A=A, lcon=S(qp.meta.lcon), ucon=S(qp.meta.ucon), lvar=S(qp.meta.lvar),
                          uvar=S(qp.meta.uvar), c0=qp.data.c0, x0=S(qp.meta.x0))
end

# ------------------------------------------------------------ linear solver plugin (linear_solver = HIPLDLSolver)
# struct madipm_ldl_opts
struct LdlOpts
    ordering::Int32
    dense_alpha::Float64
    relax::Int32
    small_front_max::Int32
    pivot_tol::Float64
    nshards::Int32
    cholesky::Int32      # ABI 0.2: Cholesky semantics (CHOLESKY with NormalKKTSystem, test/test_gpu.jl:11)
end

Base.@kwdef mutable struct HIPLDLOptions <: MadNLP.AbstractOptions
    ordering::Int32 = 4            # 0 natural, 1 AMD, 3 nested dissection, 4 the one with fewer flops
    relax::Int32 = 1
    small_front_max::Int32 = 128
    pivot_tol::Float64 = 0.0
    cholesky::Bool = false         # MadNLPGPU's cudss_algorithm = CHOLESKY counterpart
end

mutable struct HIPLDLSolver{T} <: MadNLP.AbstractLinearSolver{T}
    handle::Ptr{Cvoid}
    csc::ROCSparseMatrixCSC{T,Int32}  # aug_com: values updated in place by build_kkt!
    opt::HIPLDLOptions
    logger::MadNLP.MadNLPLogger
end

# LS(aug_com; opt) — symbolic analysis + upload (src/KKT/normalkkt.jl:113-115); either triangle
function HIPLDLSolver(csc::ROCSparseMatrixCSC{T,Int32}; opt=HIPLDLOptions(),
                      logger=MadNLP.MadNLPLogger()) where T
    colptr = Int64.(Array(csc.colPtr)) .- 1
    rowval = Int32.(Array(csc.rowVal)) .- Int32(1)
    o = Ref(LdlOpts(opt.ordering, 10.0, opt.relax, opt.small_front_max, opt.pivot_tol, Int32(1), Int32(opt.cholesky)))
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:madipm_ldl_analyze, libmadipm), Cint,
                (Int32, Ptr{Int64}, Ptr{Int32}, Ref{LdlOpts}, Ptr{Int32}, Ref{Ptr{Cvoid}}),
                size(csc, 1), colptr, rowval, o, C_NULL, h), "madipm_ldl_analyze")
    s = HIPLDLSolver{T}(h[], csc, opt, logger)
    finalizer(x -> ccall((:madipm_ldl_destroy, libmadipm), Cvoid, (Ptr{Cvoid},), x.handle), s)
    return s
end

function MadNLP.factorize!(s::HIPLDLSolver)
    GC.@preserve s check(ccall((:madipm_ldl_factorize, libmadipm), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ptr{Cvoid}),
                               s.handle, pointer(nonzeros(s.csc)), hipstream()), "madipm_ldl_factorize")
    return s                                        # rc > 0  <=>  is_factorized(s) == false
end

function MadNLP.solve!(s::HIPLDLSolver{T}, x::ROCVector{T}) where T
    GC.@preserve x check(ccall((:madipm_ldl_solve, libmadipm), Cint, (Ptr{Cvoid}, Ptr{T}, Int32, Ptr{Cvoid}),
                               s.handle, pointer(x), Int32(1), hipstream()), "madipm_ldl_solve")
    return x
end

MadIPM.is_factorized(s::HIPLDLSolver) =                       # src/utils.jl:54-62
    ccall((:madipm_ldl_is_factorized, libmadipm), Cint, (Ptr{Cvoid},), s.handle) == 1
MadNLP.is_inertia(::HIPLDLSolver) = true
function MadNLP.inertia(s::HIPLDLSolver)
    p, z, n = Ref{Int32}(0), Ref{Int32}(0), Ref{Int32}(0)
    check(ccall((:madipm_ldl_inertia, libmadipm), Cint, (Ptr{Cvoid}, Ref{Int32}, Ref{Int32}, Ref{Int32}),
                s.handle, p, z, n), "madipm_ldl_inertia")
    return (Int(p[]), Int(z[]), Int(n[]))
end
MadNLP.improve!(::HIPLDLSolver) = false
MadNLP.introduce(::HIPLDLSolver) = "madipm-hip multifrontal LDL^T (gfx950)"
MadNLP.is_supported(::Type{HIPLDLSolver}, ::Type{Float64}) = true
MadNLP.default_options(::Type{HIPLDLSolver}) = HIPLDLOptions()

# ------------------------------------------------------------ whole-solver route (native MPC driver)
# struct madipm_qp / madipm_options / madipm_stats of include/madipm_hip.h (same field order: C layout)
struct MadipmQP
    nvar::Int32; ncon::Int32; nnzh::Int64; nnzj::Int64
    c::Ptr{Float64}; c0::Float64
    Hrows::Ptr{Int32}; Hcols::Ptr{Int32}; Hvals::Ptr{Float64}
    Arows::Ptr{Int32}; Acols::Ptr{Int32}; Avals::Ptr{Float64}
    lcon::Ptr{Float64}; ucon::Ptr{Float64}; lvar::Ptr{Float64}; uvar::Ptr{Float64}
    x0::Ptr{Float64}; y0::Ptr{Float64}; minimize::Int32
end

struct MadipmOptions          # IPMOptions (src/utils.jl:69-105) + the linear solver's options
    tol::Float64; max_iter::Int32; max_wall_time::Float64; divergence_tol::Float64; scaling::Int32
    bound_push::Float64; bound_fac::Float64; bound_relax_factor::Float64
    regularization::Int32; delta_p::Float64; delta_d::Float64; delta_min::Float64
    step_rule::Int32; step_tau::Float64; max_ncorr::Int32
    mu_init::Float64; mu_min::Float64; tol_linear_solve::Float64; check_residual::Int32
    kkt_system::Int32; print_level::Int32
    ldl::LdlOpts
end

struct MadipmStats
    status::Int32; iter::Int32
    objective::Float64; dual_objective::Float64
    inf_pr::Float64; inf_du::Float64; inf_compl::Float64; mu::Float64
    total_time::Float64; linear_solver_time::Float64; init_time::Float64
    exception::Int32          # MADIPM_EXC_*: 1 SolveException, 2 solve with an unfactorized matrix
end

# rebuild an immutable struct with some fields replaced
_with(x::T; kw...) where {T} = T((haskey(kw, f) ? convert(fieldtype(T, f), kw[f]) : getfield(x, f) for f in fieldnames(T))...)

const _IPM_SCALARS = (:tol, :max_iter, :max_wall_time, :divergence_tol, :bound_push, :bound_fac,
                      :bound_relax_factor, :max_ncorr, :mu_init, :mu_min, :tol_linear_solve)
const _LDL_KEYS = (:ordering, :dense_alpha, :relax, :small_front_max, :pivot_tol, :nshards)

# load_options (src/utils.jl:121-148) onto struct madipm_options: the IPMOptions keyword names and
# types of the reference; leftovers are reported as ignored (MadNLP.print_ignored_options, l.140-142)
function madipm_options(; kwargs...)
    r = Ref{MadipmOptions}()
    ccall((:madipm_default_options, libmadipm), Cvoid, (Ref{MadipmOptions},), r)
    o = r[]
    kw = Dict{Symbol,Any}(kwargs)
    set = Dict{Symbol,Any}()
    for k in _IPM_SCALARS
        haskey(kw, k) && (set[k] = pop!(kw, k))
    end
    haskey(kw, :scaling) && (set[:scaling] = Int32(pop!(kw, :scaling)))
    haskey(kw, :check_residual) && (set[:check_residual] = Int32(pop!(kw, :check_residual)))
    if haskey(kw, :regularization)
        reg = pop!(kw, :regularization)
        if reg isa MadIPM.NoRegularization
            set[:regularization] = 0
        elseif reg isa MadIPM.FixedRegularization
            set[:regularization] = 1; set[:delta_p] = reg.delta_p; set[:delta_d] = reg.delta_d
        elseif reg isa MadIPM.AdaptiveRegularization
            set[:regularization] = 2; set[:delta_p] = reg.delta_p; set[:delta_d] = reg.delta_d
            set[:delta_min] = reg.delta_min
        else
            error("madipm_hip: unsupported regularization $(typeof(reg))")
        end
    end
    if haskey(kw, :step_rule)
        rule = pop!(kw, :step_rule)
        if rule isa MadIPM.ConservativeStep
            set[:step_rule] = 0; set[:step_tau] = rule.tau
        elseif rule isa MadIPM.AdaptiveStep
            set[:step_rule] = 1; set[:step_tau] = rule.tau_min
        elseif rule isa MadIPM.MehrotraAdaptiveStep
            set[:step_rule] = 2; set[:step_tau] = rule.gamma_f
        else
            error("madipm_hip: unsupported step rule $(typeof(rule))")
        end
    end
    if haskey(kw, :kkt_system)
        K = pop!(kw, :kkt_system)
        set[:kkt_system] = K <: MadNLP.ScaledSparseKKTSystem ? 1 : K <: MadIPM.NormalKKTSystem ? 2 :
                           K <: MadNLP.SparseKKTSystem ? 0 : error("madipm_hip: unsupported kkt_system $K")
    end
    haskey(kw, :print_level) && (set[:print_level] = Int32(pop!(kw, :print_level) <= MadNLP.INFO))
    haskey(kw, :barrier_update) && pop!(kw, :barrier_update) isa MadIPM.Mehrotra
    haskey(kw, :linear_solver) && pop!(kw, :linear_solver)   # the native route always uses the HIP LDL^T
    ldl = Dict{Symbol,Any}(k => pop!(kw, k) for k in _LDL_KEYS if haskey(kw, k))
    rethrow_error = Bool(pop!(kw, :rethrow_error, false))
    isempty(kw) || @warn "The following options are ignored: $(join(keys(kw), ", "))"
    o = _with(o; set...)
    isempty(ldl) || (o = _with(o; ldl=_with(o.ldl; ldl...)))
    return o, rethrow_error
end

struct HIPSolveException <: Exception
    code::Int32
end
Base.showerror(io::IO, e::HIPSolveException) =
    print(io, e.code == 1 ? "MadNLP.SolveException (residual check of solve_system!)" :
              "solve with an unfactorized KKT system")

"""
    madipm_hip(qp::QuadraticModel{Float64}; kwargs...) -> NamedTuple

`MPCSolver(qp; kwargs...)` + `solve!` run entirely on the GPU (src/structure.jl:79-178,
src/solver.jl:362-418), with the reference's keyword names (`IPMOptions`, src/utils.jl:69-119;
`regularization`, `step_rule`, `kkt_system` take the reference's types) plus the linear solver's
(`ordering`, `relax`, `small_front_max`, `pivot_tol`, `nshards`).  Returns the fields of
MadNLP.MadNLPExecutionStats that update_solution! fills (src/utils.jl:150-156).  An exception caught by
solve!'s catch-all (status INTERNAL_ERROR) is rethrown when `rethrow_error = true` (src/solver.jl:402).
"""
function madipm_hip(qp::QuadraticModel{Float64}; kwargs...)
    d, m = qp.data, qp.meta
    Hr, Hc = Int32.(d.H.rows) .- Int32(1), Int32.(d.H.cols) .- Int32(1)
    Ar, Ac = Int32.(d.A.rows) .- Int32(1), Int32.(d.A.cols) .- Int32(1)
    opts, rethrow_error = madipm_options(; kwargs...)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve Hr Hc Ar Ac d m begin
        q = Ref(MadipmQP(m.nvar, m.ncon, length(d.H.vals), length(d.A.vals), pointer(d.c), d.c0,
                         pointer(Hr), pointer(Hc), pointer(d.H.vals), pointer(Ar), pointer(Ac), pointer(d.A.vals),
                         pointer(m.lcon), pointer(m.ucon), pointer(m.lvar), pointer(m.uvar),
                         pointer(m.x0), pointer(m.y0), Int32(m.minimize)))
        check(ccall((:madipm_solver_create, libmadipm), Cint,
                    (Ref{MadipmQP}, Ref{MadipmOptions}, Ref{Ptr{Cvoid}}), q, Ref(opts), h), "madipm_solver_create")
    end
    st = Ref{MadipmStats}()
    try
        check(ccall((:madipm_solver_solve, libmadipm), Cint, (Ptr{Cvoid}, Ref{MadipmStats}), h[], st),
              "madipm_solver_solve")
        s = st[]
        (rethrow_error && s.status == Int32(MadNLP.INTERNAL_ERROR) && s.exception > 0) &&
            throw(HIPSolveException(s.exception))
        x, zl, zu = zeros(m.nvar), zeros(m.nvar), zeros(m.nvar)
        y, cons = zeros(m.ncon), zeros(m.ncon)
        check(ccall((:madipm_solver_get_solution, libmadipm), Cint,
                    (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                    h[], x, y, zl, zu, cons), "madipm_solver_get_solution")
        return (status = MadNLP.Status(s.status), iter = Int(s.iter), objective = s.objective,
                dual_objective = s.dual_objective, solution = x, constraints = cons, multipliers = y,
                multipliers_L = zl, multipliers_U = zu, primal_feas = s.inf_pr, dual_feas = s.inf_du,
                total_time = s.total_time, linear_solver_time = s.linear_solver_time)
    finally
        ccall((:madipm_solver_destroy, libmadipm), Cvoid, (Ptr{Cvoid},), h[])
    end
end

end # module
