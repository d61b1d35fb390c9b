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
end

Base.@kwdef mutable struct HIPLDLOptions <: MadNLP.AbstractOptions
    ordering::Int32 = 4            # 0 natural, 1 AMD, 3 nested dissection, 4 the one with fewer flops
    relax::Int32 = 1
    small_front_max::Int32 = 128
    pivot_tol::Float64 = 0.0
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
    o = Ref(LdlOpts(opt.ordering, 10.0, opt.relax, opt.small_front_max, opt.pivot_tol, Int32(1)))
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
# struct madipm_qp / madipm_options / madipm_stats of include/madipm_hip.h
struct MadipmQP
    nvar::Int32; ncon::Int32; nnzh::Int64; nnzj::Int64
    c::Ptr{Float64}; c0::Float64
    Hrows::Ptr{Int32}; Hcols::Ptr{Int32}; Hvals::Ptr{Float64}
    Arows::Ptr{Int32}; Acols::Ptr{Int32}; Avals::Ptr{Float64}
    lcon::Ptr{Float64}; ucon::Ptr{Float64}; lvar::Ptr{Float64}; uvar::Ptr{Float64}
    x0::Ptr{Float64}; y0::Ptr{Float64}; minimize::Int32
end

"""
    madipm_hip(qp::QuadraticModel{Float64}; options...) -> (status, objective, iter, x, y, zl, zu)

`MPCSolver(qp; kwargs...)` + `solve!` run entirely on the GPU (src/structure.jl:79-178,
src/solver.jl:362-418).  `options` are the fields of `struct madipm_options`, set through
`madipm_default_options` + the keyword names of `IPMOptions` (src/utils.jl:69-119).
"""
function madipm_hip(qp::QuadraticModel{Float64}; set_options! = (o -> o))
    d, m = qp.data, qp.meta
    Hr, Hc = Int32.(d.H.rows) .- Int32(1), Int32.(d.H.cols) .- Int32(1)
    Ar, Ac = Int32.(d.A.rows) .- Int32(1), Int32.(d.A.cols) .- Int32(1)
    opts = zeros(UInt8, 4096)                       # struct madipm_options, filled by the library
    ccall((:madipm_default_options, libmadipm), Cvoid, (Ptr{UInt8},), opts)
    set_options!(opts)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve Hr Hc Ar Ac d m opts begin
        q = Ref(MadipmQP(m.nvar, m.ncon, length(d.H.vals), length(d.A.vals), pointer(d.c), d.c0,
                         pointer(Hr), pointer(Hc), pointer(d.H.vals), pointer(Ar), pointer(Ac), pointer(d.A.vals),
                         pointer(m.lcon), pointer(m.ucon), pointer(m.lvar), pointer(m.uvar),
                         pointer(m.x0), pointer(m.y0), Int32(m.minimize)))
        check(ccall((:madipm_solver_create, libmadipm), Cint, (Ref{MadipmQP}, Ptr{UInt8}, Ref{Ptr{Cvoid}}),
                    q, opts, h), "madipm_solver_create")
    end
    stats = zeros(UInt8, 256)                       # struct madipm_stats
    try
        check(ccall((:madipm_solver_solve, libmadipm), Cint, (Ptr{Cvoid}, Ptr{UInt8}), h[], stats), "madipm_solver_solve")
        x, zl, zu = zeros(m.nvar), zeros(m.nvar), zeros(m.nvar)
        y = zeros(m.ncon)
        check(ccall((:madipm_solver_get_solution, libmadipm), Cint,
                    (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                    h[], x, y, zl, zu, C_NULL), "madipm_solver_get_solution")
        status = reinterpret(Int32, stats[1:4])[1]
        objective = reinterpret(Float64, stats[9:16])[1]
        iter = reinterpret(Int32, stats[5:8])[1]
        return (status, objective, iter, x, y, zl, zu)
    finally
        ccall((:madipm_solver_destroy, libmadipm), Cvoid, (Ptr{Cvoid},), h[])
    end
end

end # module
