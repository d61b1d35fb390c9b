# ROCArray methods of MadIPM / MadNLP / NLPModels over libmadipm_hip.so (include/madipm_hip.h).
#
# Counterpart of the reference's ext/MadIPMCUDAExt/cuda_wrapper.jl: every kernel of that file is
# replaced by a C-ABI entry point of csrc/kkt.hip (hand-written gfx950 HIP, fixed summation orders).
# The C-ABI is 0-based; Julia's sparse device matrices are 1-based, so index arrays are shifted once
# (structure arrays never change after construction: `zero_based` caches the shifted copy per array)
# while value arrays are passed through untouched and read live.
#
# Not executed in this repository (no Julia toolchain in the image); the Python mirror
# madipm_amd/rocm_wrapper.py binds the same symbols and is what tests/test_kkt_ops_gpu.py runs.

const libmadipm = get(ENV, "MADIPM_HIP_LIB", joinpath(@__DIR__, "..", "..", "madipm_amd", "lib", "libmadipm_hip.so"))

function check(rc::Integer, what::AbstractString="libmadipm_hip")
    rc < 0 && error(what, ": ", unsafe_string(ccall((:madipm_last_error, libmadipm), Cstring, ())))
    return Int(rc)
end

hipstream() = AMDGPU.stream().stream                 # hipStream_t of the task-local stream

# Per-array caches keyed by object IDENTITY (objectid), never by content: hashing a device array would
# read it element by element from the host.  The entry is dropped by a finalizer on the key array.
function cached!(f, cache::Dict{UInt,Any}, x)
    id = objectid(x)
    v = get(cache, id, nothing)
    v === nothing || return v
    v = f()
    cache[id] = v
    finalizer(_ -> delete!(cache, id), x)
    return v
end

# 0-based copies of 1-based index arrays (structure arrays: never change after construction)
const ZB = Dict{UInt,Any}()
zero_based(x::ROCVector{Ti}) where {Ti<:Integer} = cached!(() -> x .- one(Ti), ZB, x)

# ------------------------------------------------------------ transfer!  (cuda_wrapper.jl:4-24)
mutable struct TransferPlan
    handle::Ptr{Cvoid}
    nsrc::Int
    ndest::Int
end
const PLANS = Dict{UInt,Any}()

function transfer_plan(map::ROCVector{Int}, ndest::Int)
    p = get(PLANS, objectid(map), nothing)
    (p !== nothing && p.ndest == ndest) && return p
    hmap = Int64.(Array(map)) .- 1                    # 0-based, host; counting-sorted by the library
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:madipm_transfer_create, libmadipm), Cint, (Int64, Ptr{Int64}, Int32, Int64, Ref{Ptr{Cvoid}}),
                length(hmap), hmap, Int32(0), ndest, h), "madipm_transfer_create")
    p = TransferPlan(h[], length(hmap), ndest)
    finalizer(q -> ccall((:madipm_transfer_destroy, libmadipm), Cvoid, (Ptr{Cvoid},), q.handle), p)
    p0 = get(PLANS, objectid(map), nothing)
    PLANS[objectid(map)] = p
    p0 === nothing && finalizer(_ -> delete!(PLANS, objectid(map)), map)
    return p
end

function MadNLP.transfer!(dest::ROCSparseMatrixCSC{Tv}, src::MadNLP.SparseMatrixCOO{Tv},
                          map::ROCVector{Int}) where {Tv<:Float64}
    # dest .= 0; dest[map[k]] += src[k], each entry summed in ascending k (deterministic)
    p = transfer_plan(map, length(nonzeros(dest)))
    GC.@preserve dest src check(ccall((:madipm_transfer, libmadipm), Cint,
                                      (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Cvoid}),
                                      p.handle, pointer(nonzeros(dest)), pointer(src.V), hipstream()), "madipm_transfer")
    return
end

function MadNLP.compress_hessian!(kkt::MadNLP.SparseKKTSystem{T,VT,MT}) where {T,VT,MT<:ROCSparseMatrixCSC{T,Int32}}
    MadNLP.transfer!(kkt.hess_com, kkt.hess_raw, kkt.hess_csc_map)
end

# ------------------------------------------------------------ compress_jacobian!  (cuda_wrapper.jl:32-41)
function MadNLP.compress_jacobian!(kkt::MadIPM.NormalKKTSystem{T,VT,MT}) where {T,VT,MT<:ROCSparseMatrixCSC{T,Int32}}
    n_slack = length(kkt.ind_ineq)
    map0 = zero_based(kkt.A_csr_map)
    GC.@preserve kkt map0 check(ccall((:madipm_compress_jacobian, libmadipm), Cint,
                                      (Ptr{Float64}, Int64, Int32, Ptr{Int64}, Ptr{Float64}, Ptr{Cvoid}),
                                      pointer(kkt.A.V), length(kkt.A.V), Int32(n_slack), pointer(map0),
                                      pointer(kkt.AT.nzVal), hipstream()), "madipm_compress_jacobian")
    return
end

# ------------------------------------------------------------ SpMV operator  (cuda_wrapper.jl:43-94)
mutable struct MadIPMOperator{T,M} <: AbstractMatrix{T}
    type::Type{T}
    m::Int
    n::Int
    A::M
    transa::Char
    handle::Ptr{Cvoid}
    rp0::ROCVector{Int32}                            # 0-based structure (values of A read live)
    ci0::ROCVector{Int32}
end

Base.eltype(A::MadIPMOperator{T}) where T = T
Base.size(A::MadIPMOperator) = (A.m, A.n)
SparseArrays.nnz(A::MadIPMOperator) = nnz(A.A)

function MadIPMOperator(A::ROCSparseMatrixCSR{T,Int32}; transa::Char='N', symmetric::Bool=false) where T<:Float64
    m, n = size(A)
    rp0, ci0 = A.rowPtr .- Int32(1), A.colVal .- Int32(1)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve A rp0 ci0 check(ccall((:madipm_spmv_create, libmadipm), Cint,
                                       (Int32, Int32, Int64, Ptr{Int32}, Ptr{Int32}, Ptr{Float64}, UInt8, Int32,
                                        Ref{Ptr{Cvoid}}),
                                       m, n, nnz(A), pointer(rp0), pointer(ci0), pointer(A.nzVal), UInt8(transa),
                                       Int32(symmetric), h), "madipm_spmv_create")
    op = MadIPMOperator{T,typeof(A)}(T, m, n, A, transa, h[], rp0, ci0)
    finalizer(o -> ccall((:madipm_spmv_destroy, libmadipm), Cvoid, (Ptr{Cvoid},), o.handle), op)
    return op
end
MadIPMOperator(A::ROCSparseMatrixCSC; kw...) = MadIPMOperator(ROCSparseMatrixCSR(A); kw...)
MadIPMOperator(A::ROCSparseMatrixCOO; kw...) = MadIPMOperator(ROCSparseMatrixCSR(A); kw...)

function LinearAlgebra.mul!(y::ROCVector{T}, A::MadIPMOperator{T}, x::ROCVector{T}, alpha::Number=one(T),
                            beta::Number=zero(T)) where T<:Float64
    GC.@preserve A x y check(ccall((:madipm_spmv_apply, libmadipm), Cint,
                                   (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Float64, Float64, Ptr{Cvoid}),
                                   A.handle, pointer(x), pointer(y), Float64(alpha), Float64(beta), hipstream()),
                             "madipm_spmv_apply")
    return y
end

# ------------------------------------------------------------ coo_to_csr  (cuda_wrapper.jl:96-106)
function MadIPM.coo_to_csr(n_rows, n_cols, Ai::ROCVector{Ti}, Aj::ROCVector{Ti}, Ax::ROCVector{Tv}) where {Tv,Ti}
    @assert length(Ai) == length(Aj) == length(Ax)
    nz = length(Ai)
    Ai0, Aj0 = Int32.(Ai) .- Int32(1), Int32.(Aj) .- Int32(1)
    Bp, Bj, Bx = ROCVector{Int32}(undef, n_rows + 1), ROCVector{Int32}(undef, nz), ROCVector{Float64}(undef, nz)
    # columns sorted within a row: the layout the reference's sparse(...; fmt=:csr) produces
    Axf = Float64.(Ax)
    GC.@preserve Ai0 Aj0 Axf Bp Bj Bx check(ccall((:madipm_coo_to_csr, libmadipm), Cint,
        (Int32, Int32, Int64, Ptr{Int32}, Ptr{Int32}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32}, Ptr{Float64}, Int32, Ptr{Cvoid}),
        n_rows, n_cols, nz, pointer(Ai0), pointer(Aj0), pointer(Axf), pointer(Bp), pointer(Bj), pointer(Bx),
        Int32(1), hipstream()), "madipm_coo_to_csr")
    return (Ti.(Bp .+ Int32(1)), Ti.(Bj .+ Int32(1)), Tv.(Bx))
end

# ------------------------------------------------------------ normal equations  (cuda_wrapper.jl:108-234)
function MadIPM.assemble_normal_system!(n_rows, n_cols, Jtp::ROCArray{Ti}, Jtj::ROCArray{Ti}, Jtx::ROCArray{Tv},
                                        Cp::ROCArray{Ti}, Cj::ROCArray{Ti}, Cx::ROCArray{Tv},
                                        Dx::ROCArray{Tv}) where {Ti<:Int32,Tv<:Float64}
    Jtp0, Jtj0, Cp0, Cj0 = zero_based(Jtp), zero_based(Jtj), zero_based(Cp), zero_based(Cj)
    GC.@preserve Jtp0 Jtj0 Cp0 Cj0 Jtx Cx Dx check(ccall((:madipm_assemble_normal_system, libmadipm), Cint,
        (Int32, Int32, Ptr{Int32}, Ptr{Int32}, Ptr{Float64}, Ptr{Int32}, Ptr{Int32}, Ptr{Float64}, Ptr{Float64}, Ptr{Cvoid}),
        n_rows, n_cols, pointer(Jtp0), pointer(Jtj0), pointer(Jtx), pointer(Cp0), pointer(Cj0), pointer(Cx),
        pointer(Dx), hipstream()), "madipm_assemble_normal_system")
    return
end

function MadIPM.build_normal_system(n_rows, n_cols, Jtp::ROCVector{Ti}, Jtj::ROCVector{Ti}) where {Ti}
    Jp, Jj = Int32.(Array(Jtp)) .- Int32(1), Int32.(Array(Jtj)) .- Int32(1)
    Cp = zeros(Int32, n_rows + 1)
    nz = Ref{Int64}(0)
    check(ccall((:madipm_build_normal_system, libmadipm), Cint,
                (Int32, Int32, Ptr{Int32}, Ptr{Int32}, Ptr{Int32}, Ptr{Int32}, Int64, Ref{Int64}),
                n_rows, n_cols, Jp, Jj, Cp, C_NULL, 0, nz), "madipm_build_normal_system")
    Cj = zeros(Int32, nz[])
    check(ccall((:madipm_build_normal_system, libmadipm), Cint,
                (Int32, Int32, Ptr{Int32}, Ptr{Int32}, Ptr{Int32}, Ptr{Int32}, Int64, Ref{Int64}),
                n_rows, n_cols, Jp, Jj, Cp, Cj, nz[], nz), "madipm_build_normal_system")
    return (ROCVector{Ti}(Cp .+ Int32(1)), ROCVector{Ti}(Cj .+ Int32(1)))
end

MadIPM.sparse_csc_format(::Type{<:ROCArray}) = ROCSparseMatrixCSC
MadIPM._colptr(A::ROCSparseMatrixCSC) = A.colPtr
MadIPM._rowval(A::ROCSparseMatrixCSC) = A.rowVal
MadIPM._nzval(A::ROCSparseMatrixCSC) = A.nzVal
