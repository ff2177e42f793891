# Julia ccall shim over libsmlu.so.  No Julia in the image: tests/test_julia_shim.py checks it
# statically against include/smlu.h (struct layout, constructor arity, every ccall'd symbol and
# its argument count).  See INTEGRATION.md.
module SharedMemSparseLU

export ParallelSparseLU, cleanup_ParallelSparseLU!, allocate_shared

using LinearAlgebra, SparseArrays, Libdl
import LinearAlgebra: ldiv!, lu!
import MPI                                     # declared by the reference (Project.toml:8)

const libsmlu = get(ENV, "SMLU_LIB", joinpath(@__DIR__, "..", "deps", "libsmlu.so"))

# entry point chosen at run time (ccall's literal (name, lib) form needs a constant name)
fnptr(name::Symbol) = Libdl.dlsym(Libdl.dlopen(libsmlu), name)

# must match `smlu_opts` in include/smlu.h field for field
mutable struct SmluOpts
    chunk_size::Int64; index_base::Int32; ordering::Int32; grid::NTuple{3,Int64}
    scale::Int32; relax::Int32; pivot_tol::Float64; diag_pivot_tol::Float64
    device::Int32; profile::Int32; leaf_size::Int64; use_mfma::Int32; refine::Int32; vendor_gemm::Int32
end
function default_opts()
    o = SmluOpts(0, 0, 0, (0, 0, 0), 0, 0, 0.0, 0.0, 0, 0, 0, 0, 0, 0)
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

# Tf in (Float64, ComplexF64), Ti in (Int64, Int32): the reference is generic in both
# (src/SharedMemSparseLU.jl:43, :64; SURVEY §8f-4).  Int32 indices go through smlu_create_i32
# (real) or are widened here (complex); complex values go through smlu_create_z as interleaved
# (re, im) doubles -- the memory layout of Vector{ComplexF64}.
const SmluFloat = Union{Float64,ComplexF64}
const SmluInt = Union{Int64,Int32}

function ParallelSparseLU(A::SparseMatrixCSC{Tf,Ti}, chunk_size=nothing) where {Tf<:SmluFloat,Ti<:SmluInt}
    chunk_size = min(something(chunk_size, 8), A.n)           # :67-72
    o = default_opts(); o.chunk_size = chunk_size
    h = Ref{Ptr{Cvoid}}(C_NULL)
    if Tf === ComplexF64
        rc = ccall((:smlu_create_z, libsmlu), Int32,
                   (Int64, Ptr{Int64}, Ptr{Int64}, Ptr{ComplexF64}, Ref{SmluOpts}, Ref{Ptr{Cvoid}}),
                   A.n, Vector{Int64}(A.colptr), Vector{Int64}(A.rowval), A.nzval, o, h)
    elseif Ti === Int32
        rc = ccall((:smlu_create_i32, libsmlu), Int32,
                   (Int64, Ptr{Int32}, Ptr{Int32}, Ptr{Float64}, Ref{SmluOpts}, Ref{Ptr{Cvoid}}),
                   A.n, A.colptr, A.rowval, A.nzval, o, h)
    else
        rc = ccall((:smlu_create, libsmlu), Int32,
                   (Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Ref{SmluOpts}, Ref{Ptr{Cvoid}}),
                   A.n, A.colptr, A.rowval, A.nzval, o, h)
    end
    if rc == 1 && h[] != C_NULL                   # singular: free the handle, then throw
        col = ccall((:smlu_last_error_col, libsmlu), Int64, (Ptr{Cvoid},), h[])
        ccall((:smlu_destroy, libsmlu), Cvoid, (Ptr{Cvoid},), h[])
        throw(SingularException(col + 1))
    end
    check(rc, h[])
    F = ParallelSparseLU{Tf,Ti}(A.m, A.n, h[], copy(A.colptr), copy(A.rowval), chunk_size)
    finalizer(cleanup_ParallelSparseLU!, F)
    return F
end

# Optional: hand UMFPACK's own analysis over so that pivot order and L/U pattern match it by
# construction (SURVEY §8f-1, §8(b)): the reference's lu(A) (:74) and its L, U, p, q, Rs
# extraction (:75-77, :93-94).  The library checks the pattern against the structural fill of
# (Rs.*A)[p, q] and exports F.L / F.U on exactly that pattern.
function ParallelSparseLU_umfpack(A::SparseMatrixCSC{Float64,Ti}, chunk_size=nothing) where {Ti<:SmluInt}
    U = lu(A)
    FL = U.L; FU = U.U
    o = default_opts(); o.chunk_size = min(something(chunk_size, 8), A.n); h = Ref{Ptr{Cvoid}}(C_NULL)
    rc = ccall((:smlu_create_with_pivots, libsmlu), Int32,
               (Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Ptr{Int64}, Ptr{Int64},
                Ptr{Float64}, Ptr{Int64}, Ptr{Int64}, Ptr{Int64}, Ptr{Int64}, Ref{SmluOpts}, Ref{Ptr{Cvoid}}),
               A.n, Vector{Int64}(A.colptr), Vector{Int64}(A.rowval), A.nzval,
               Vector{Int64}(U.p), Vector{Int64}(U.q), U.Rs,
               Vector{Int64}(FL.colptr), Vector{Int64}(FL.rowval),
               Vector{Int64}(FU.colptr), Vector{Int64}(FU.rowval), o, h)
    check(rc, h[])
    F = ParallelSparseLU{Float64,Ti}(A.m, A.n, h[], copy(A.colptr), copy(A.rowval), o.chunk_size)
    finalizer(cleanup_ParallelSparseLU!, F)
    return F
end

# One process per GPU (the rank split the reference only sketches, :107, :128; MPI is its declared
# dependency, Project.toml:8).  Collective over `comm`: rank 0 creates the RCCL unique id, MPI
# broadcasts the 128 bytes, every rank builds its part of the partition on its node-local GPU and
# the library moves the blocks itself over RCCL/xGMI.  lu! and ldiv! below are then collective too
# (every rank calls them with the same values / right-hand side; x comes back complete everywhere).
function ParallelSparseLU(A::SparseMatrixCSC{Float64,Int64}, comm::MPI.Comm, chunk_size=nothing)
    rank = MPI.Comm_rank(comm); nranks = MPI.Comm_size(comm)
    id = zeros(UInt8, 128)
    rank == 0 && check(ccall((:smlu_rccl_unique_id, libsmlu), Int32, (Ptr{UInt8},), id), C_NULL)
    MPI.Bcast!(id, 0, comm)
    o = default_opts(); o.chunk_size = min(something(chunk_size, 8), A.n)
    o.device = MPI.Comm_rank(MPI.Comm_split_type(comm, MPI.COMM_TYPE_SHARED, rank))   # node-local GPU
    h = Ref{Ptr{Cvoid}}(C_NULL)
    rc = ccall((:smlu_dist_create_rccl, libsmlu), Int32,
               (Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Ref{SmluOpts}, Int32, Int32, Ptr{UInt8},
                Ref{Ptr{Cvoid}}),
               A.n, A.colptr, A.rowval, A.nzval, o, rank, nranks, id, h)
    check(rc, h[])
    F = ParallelSparseLU{Float64,Int64}(A.m, A.n, h[], copy(A.colptr), copy(A.rowval), o.chunk_size)
    finalizer(cleanup_ParallelSparseLU!, F)
    return F
end

function lu!(F::ParallelSparseLU{Tf,Ti}, A::SparseMatrixCSC{Tf,Ti}) where {Tf,Ti}   # :245-279
    z = Tf === ComplexF64
    if A.colptr == F.colptr && A.rowval == F.rowval
        rc = ccall(fnptr(z ? :smlu_refactor_z : :smlu_refactor), Int32, (Ptr{Cvoid}, Ptr{Tf}),
                   F.handle, A.nzval)
    else                                                                          # :265-273
        rc = ccall(fnptr(z ? :smlu_refactor_csc_z : :smlu_refactor_csc), Int32,
                   (Ptr{Cvoid}, Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Tf}),
                   F.handle, A.n, Vector{Int64}(A.colptr), Vector{Int64}(A.rowval), A.nzval)
        F.colptr = copy(A.colptr); F.rowval = copy(A.rowval)
    end
    check(rc, F.handle)
    return nothing
end

function ldiv!(x::AbstractVecOrMat, F::ParallelSparseLU{Tf}, b::AbstractVecOrMat) where {Tf}   # :286-342
    @boundscheck F.m == F.n || throw(DimensionMismatch("`F` is not square: F.m=$(F.m), F.n=$(F.n)"))
    @boundscheck size(x, 1) == F.n || throw(DimensionMismatch("`x` does not have same size as F: length(x)=$(length(x)), F.n=$(F.n)"))
    @boundscheck size(b, 1) == F.n || throw(DimensionMismatch("`b` does not have same size as F: length(b)=$(length(b)), F.n=$(F.n)"))
    bb = b isa Array{Tf} ? b : Array{Tf}(b)
    xx = x isa Array{Tf} ? x : similar(bb)
    if ndims(b) == 1
        check(ccall((:smlu_solve, libsmlu), Int32, (Ptr{Cvoid}, Ptr{Tf}, Ptr{Tf}), F.handle, bb, xx), F.handle)
    else                                       # several right-hand sides: one batched call
        ld = (Tf === ComplexF64 ? 2 : 1) * F.n  # leading dimension in doubles
        check(ccall((:smlu_solve_multi, libsmlu), Int32,
                    (Ptr{Cvoid}, Int64, Ptr{Tf}, Int64, Ptr{Tf}, Int64),
                    F.handle, size(b, 2), bb, ld, xx, ld), F.handle)
    end
    xx === x || copyto!(x, xx)
    return x
end

function _trisolve!(upper::Bool, F::ParallelSparseLU{Tf}, x::AbstractVector) where {Tf}
    xx = x isa Vector{Tf} ? x : Vector{Tf}(x)
    check(ccall(fnptr(upper ? :smlu_rsolve : :smlu_lsolve), Int32, (Ptr{Cvoid}, Ptr{Tf}), F.handle, xx),
          F.handle)
    xx === x || copyto!(x, xx)
    return nothing
end
lsolve!(F::ParallelSparseLU, x) = _trisolve!(false, F, x)                          # :349
rsolve!(F::ParallelSparseLU, x) = _trisolve!(true, F, x)                           # :374

# Optional parity mode: the reference's own dense-chunk layout (:101-243) on the GPU, refilled
# after each lu! (:265-276); ldiv! through it runs lsolve!/rsolve! chunk by chunk (:349-392).
chunked_setup!(F::ParallelSparseLU) = check(ccall((:smlu_chunked_setup, libsmlu), Int32,
    (Ptr{Cvoid}, Int64), F.handle, F.chunk_size), F.handle)
function chunked_ldiv!(x::AbstractVector, F::ParallelSparseLU{Tf}, b::AbstractVector) where {Tf}
    length(x) == length(b) == F.n || throw(DimensionMismatch("x, b and F sizes differ"))
    bb = Vector{Tf}(b); xx = Vector{Tf}(undef, F.n)
    check(ccall((:smlu_chunked_ldiv, libsmlu), Int32, (Ptr{Cvoid}, Ptr{Tf}, Ptr{Tf}),
                F.handle, bb, xx), F.handle)
    copyto!(x, xx)
end

function Base.getproperty(F::ParallelSparseLU{Tf,Ti}, s::Symbol) where {Tf,Ti}     # :45-52
    s in (:L, :U, :p, :q, :Rs) || return getfield(F, s)
    h = getfield(F, :handle)
    n = Int64(getfield(F, :n)); nl = Ref{Int64}(0); nu = Ref{Int64}(0)
    # ComplexF64: the complex factors, folded from the real-equivalent ones (smlu_get_factors_z)
    z = Tf === ComplexF64
    check(ccall(fnptr(z ? :smlu_get_sizes_z : :smlu_get_sizes), Int32,
                (Ptr{Cvoid}, Ptr{Int64}, Ref{Int64}, Ref{Int64}), h, C_NULL, nl, nu), h)
    Lp = Vector{Int64}(undef, n + 1); Li = Vector{Int64}(undef, nl[]); Lx = Vector{Tf}(undef, nl[])
    Up = Vector{Int64}(undef, n + 1); Ui = Vector{Int64}(undef, nu[]); Ux = Vector{Tf}(undef, nu[])
    p = Vector{Int64}(undef, n); q = Vector{Int64}(undef, n); Rs = Vector{Float64}(undef, n)
    check(ccall(fnptr(z ? :smlu_get_factors_z : :smlu_get_factors), Int32,
                (Ptr{Cvoid}, Ptr{Int64}, Ptr{Int64}, Ptr{Tf}, Ptr{Int64}, Ptr{Int64},
                 Ptr{Tf}, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}),
                h, Lp, Li, Lx, Up, Ui, Ux, p, q, Rs), h)
    s === :L && return SparseMatrixCSC{Tf,Ti}(n, n, Vector{Ti}(Lp), Vector{Ti}(Li), Lx)   # L::SparseMatrixCSC{Tf,Ti}
    s === :U && return SparseMatrixCSC{Tf,Ti}(n, n, Vector{Ti}(Up), Vector{Ti}(Ui), Ux)
    s === :p && return Vector{Ti}(p)           # p::Vector{Ti}, q::Vector{Ti} as the reference (:49-50)
    s === :q && return Vector{Ti}(q)
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
