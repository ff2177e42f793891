"""smlu — MI355X-native (gfx950) sparse LU refactorize/solve, a drop-in for the hot path of
SharedMemSparseLU.jl (ParallelSparseLU / lu! / ldiv!).  Host symbolic analysis + HIP kernels
in libsmlu.so (C-ABI: include/smlu.h); this package is the Python mirror of the Julia API."""
from ._lib import build, lib, default_opts, LIB_PATH  # noqa: F401
from .api import (ParallelSparseLU, lu_, ldiv_, lsolve_, rsolve_,  # noqa: F401
                  chunked_setup, chunked_ldiv_, cleanup_ParallelSparseLU_, allocate_shared, DimensionMismatch,
                  SingularException, SmluError)
from .plan import Plan  # noqa: F401
from .dist import DistributedSparseLU  # noqa: F401

__all__ = ["ParallelSparseLU", "lu_", "ldiv_", "lsolve_", "rsolve_", "chunked_setup", "chunked_ldiv_",
           "cleanup_ParallelSparseLU_",
           "allocate_shared", "DimensionMismatch", "SingularException", "SmluError", "Plan", "DistributedSparseLU", "build",
           "lib"]
