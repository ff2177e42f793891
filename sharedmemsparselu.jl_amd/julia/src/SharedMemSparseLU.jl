# Julia ccall shim over libsmlu.so (untested here: no Julia in the image). See INTEGRATION.md.
module SharedMemSparseLU

export ParallelSparseLU, cleanup_ParallelSparseLU!, allocate_shared

using LinearAlgebra, SparseArrays
import LinearAlgebra: ldiv!, lu!

const libsmlu = get(ENV, "SMLU_LIB", joinpath(@__DIR__, "..", "deps", "libsmlu.so"))

# must match `smlu_opts` in include/smlu.h field for field
mutable struct SmluOpts
    chunk_size::Int64; index_base::Int32; ordering::Int32; grid::NTuple{3,Int64}
    scale::Int32; relax::Int32; pivot_tol::Float64; diag_pivot_tol::Float64
    device::Int32; profile::Int32; leaf_size::Int64; use_mfma::Int32; refine::Int32; vendor_gemm::Int32
end
function default_opts()
    o = SmluOpts(0, 0, 0, (0, 0, 0), 0, 0, 0.0, 0.0, 0, 0, 0, 0, 0)
    ccall((:smlu_default_opts, libsmlu), Cvoid, (Ref{SmluOpts},), o)
    return o                                   # index_base = 1: Julia's 1-based CSC as is
end

struct SmluError <: Exception; code::Int32; msg::String; end
function check(rc, h)
    rc == 0 && return
    msg = unsafe_string(ccall((:smlu_last_error_string, libsmlu), Cstring, (Ptr{Cvoid},), h))
    if rc == 1                                 # SMLU_SINGULAR, as UMFPACK's check=true
        col = ccall((:smlu_last_error_col, libsmlu), Int64, (Ptr{Cvoid},), h)
        throw(SingularException(col + 1))
    end
    rc < 0 && throw(SmluError(rc, msg))
end

mutable struct ParallelSparseLU{Tf,Ti}
    m::Ti; n::Ti
    handle::Ptr{Cvoid}
    colptr::Vector{Ti}; rowval::Vector{Ti}
    chunk_size::Ti
end

function ParallelSparseLU(A::SparseMatrixCSC{Float64,Int64}, chunk_size=nothing)
    chunk_size = min(something(chunk_size, 8), A.n)           # :67-72
    o = default_opts(); o.chunk_size = chunk_size
    h = Ref{Ptr{Cvoid}}(C_NULL)
    rc = ccall((:smlu_create, libsmlu), Int32,
               (Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Ref{SmluOpts}, Ref{Ptr{Cvoid}}),
               A.n, A.colptr, A.rowval, A.nzval, o, h)
    check(rc, h[])
    F = ParallelSparseLU{Float64,Int64}(A.m, A.n, h[], copy(A.colptr), copy(A.rowval), chunk_size)
    finalizer(cleanup_ParallelSparseLU!, F)
    return F
end

# Optional: hand UMFPACK's own analysis over so that pivot order matches it by construction.
function ParallelSparseLU_umfpack(A::SparseMatrixCSC{Float64,Int64})
    U = lu(A)
    o = default_opts(); h = Ref{Ptr{Cvoid}}(C_NULL)
    rc = ccall((:smlu_create_with_pivots, libsmlu), Int32,
               (Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Ptr{Int64}, Ptr{Int64},
                Ptr{Float64}, Ref{SmluOpts}, Ref{Ptr{Cvoid}}),
               A.n, A.colptr, A.rowval, A.nzval, U.p, U.q, U.Rs, o, h)
    check(rc, h[])
    return ParallelSparseLU{Float64,Int64}(A.m, A.n, h[], copy(A.colptr), copy(A.rowval), 8)
end

function lu!(F::ParallelSparseLU{Tf,Ti}, A::SparseMatrixCSC{Tf,Ti}) where {Tf,Ti}   # :245-279
    if A.colptr == F.colptr && A.rowval == F.rowval
        rc = ccall((:smlu_refactor, libsmlu), Int32, (Ptr{Cvoid}, Ptr{Float64}), F.handle, A.nzval)
    else                                                                          # :265-273
        rc = ccall((:smlu_refactor_csc, libsmlu), Int32,
                   (Ptr{Cvoid}, Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}),
                   F.handle, A.n, A.colptr, A.rowval, A.nzval)
        F.colptr = copy(A.colptr); F.rowval = copy(A.rowval)
    end
    check(rc, F.handle)
    return nothing
end

function ldiv!(x::AbstractVector, F::ParallelSparseLU, b::AbstractVector)        # :286-342
    @boundscheck F.m == F.n || throw(DimensionMismatch("`F` is not square: F.m=$(F.m), F.n=$(F.n)"))
    @boundscheck length(x) == F.n || throw(DimensionMismatch("`x` does not have same size as F: length(x)=$(length(x)), F.n=$(F.n)"))
    @boundscheck length(b) == F.n || throw(DimensionMismatch("`b` does not have same size as F: length(b)=$(length(b)), F.n=$(F.n)"))
    bb = b isa Vector{Float64} ? b : Vector{Float64}(b)
    xx = x isa Vector{Float64} ? x : similar(bb)
    check(ccall((:smlu_solve, libsmlu), Int32, (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}),
                F.handle, bb, xx), F.handle)
    xx === x || copyto!(x, xx)
    return x
end

lsolve!(F::ParallelSparseLU, x) = (check(ccall((:smlu_lsolve, libsmlu), Int32,
    (Ptr{Cvoid}, Ptr{Float64}), F.handle, x), F.handle); nothing)                   # :349
rsolve!(F::ParallelSparseLU, x) = (check(ccall((:smlu_rsolve, libsmlu), Int32,
    (Ptr{Cvoid}, Ptr{Float64}), F.handle, x), F.handle); nothing)                   # :374

function Base.getproperty(F::ParallelSparseLU, s::Symbol)                           # :45-52
    s in (:L, :U, :p, :q, :Rs) || return getfield(F, s)
    n = getfield(F, :n); nl = Ref{Int64}(0); nu = Ref{Int64}(0)
    h = getfield(F, :handle)
    check(ccall((:smlu_get_sizes, libsmlu), Int32, (Ptr{Cvoid}, Ptr{Int64}, Ref{Int64}, Ref{Int64}),
                h, C_NULL, nl, nu), h)
    Lp = Vector{Int64}(undef, n + 1); Li = Vector{Int64}(undef, nl[]); Lx = Vector{Float64}(undef, nl[])
    Up = Vector{Int64}(undef, n + 1); Ui = Vector{Int64}(undef, nu[]); Ux = Vector{Float64}(undef, nu[])
    p = Vector{Int64}(undef, n); q = Vector{Int64}(undef, n); Rs = Vector{Float64}(undef, n)
    check(ccall((:smlu_get_factors, libsmlu), Int32,
                (Ptr{Cvoid}, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Ptr{Int64}, Ptr{Int64},
                 Ptr{Float64}, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}),
                h, Lp, Li, Lx, Up, Ui, Ux, p, q, Rs), h)
    s === :L && return SparseMatrixCSC(n, n, Lp, Li, Lx)
    s === :U && return SparseMatrixCSC(n, n, Up, Ui, Ux)
    s === :p && return p
    s === :q && return q
    return Rs
end

function cleanup_ParallelSparseLU!(F::ParallelSparseLU)                             # :31
    h = getfield(F, :handle)
    h == C_NULL || ccall((:smlu_destroy, libsmlu), Cvoid, (Ptr{Cvoid},), h)
    setfield!(F, :handle, C_NULL)
    return nothing
end

allocate_shared(T, dims...) = zeros(T, dims...)   # exported but undefined in the reference

end
