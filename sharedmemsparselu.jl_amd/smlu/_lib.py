"""ctypes binding of libsmlu.so (C-ABI declared in include/smlu.h).

No torch types cross this boundary: plain pointers and int64 sizes, as a Julia ``ccall``
shim would bind them.  The product never falls back to the CPU: if the
library is missing, or no gfx950 device is visible, calls fail loudly.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # sharedmemsparselu.jl_amd/
LIB_PATH = os.environ.get("SMLU_LIB") or os.path.join(_PKG, "libsmlu.so")   # SMLU_LIB: dev variants

i64 = ctypes.c_int64
i32 = ctypes.c_int32
f64 = ctypes.c_double
i64p = ctypes.POINTER(ctypes.c_int64)
f64p = ctypes.POINTER(ctypes.c_double)
vp = ctypes.c_void_p

SMLU_OK = 0
SMLU_SINGULAR = 1
SMLU_PIVOT_WEAK = 2
SMLU_ERR_ARG = -1
SMLU_ERR_PATTERN = -2
SMLU_ERR_ALLOC = -3
SMLU_ERR_HIP = -4
SMLU_ERR_NODEVICE = -5
SMLU_ERR_STATE = -6

ORDER_AUTO, ORDER_NATURAL, ORDER_GEOMETRIC_ND, ORDER_GRAPH_ND, ORDER_GIVEN, ORDER_AMD = range(6)


class SmluOpts(ctypes.Structure):
    _fields_ = [
        ("chunk_size", i64),
        ("index_base", i32),
        ("ordering", i32),
        ("grid", i64 * 3),
        ("scale", i32),
        ("relax", i32),
        ("pivot_tol", f64),
        ("diag_pivot_tol", f64),
        ("device", i32),
        ("profile", i32),
        ("leaf_size", i64),
        ("use_mfma", i32),
        ("refine", i32),
        ("vendor_gemm", i32),
    ]


# exported symbols and their signatures (restype, argtypes); the CPU test-suite checks that
# every function declared in include/smlu.h is present here and in the .so
SIGNATURES = {
    "smlu_default_opts": (None, [ctypes.POINTER(SmluOpts)]),
    "smlu_create": (i32, [i64, vp, vp, vp, ctypes.POINTER(SmluOpts), ctypes.POINTER(vp)]),
    "smlu_create_with_pivots": (i32, [i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.POINTER(SmluOpts),
                                      ctypes.POINTER(vp)]),
    "smlu_refactor": (i32, [vp, vp]),
    "smlu_refactor_device": (i32, [vp, vp]),
    "smlu_set_stream": (i32, [vp, vp]),
    "smlu_dev_front_hash": (i32, [vp, vp]),
    "smlu_dev_front_values": (i32, [vp, i64, vp]),
    "smlu_dev_front_offsets": (i32, [vp, vp]),
    "smlu_dev_copy": (i32, [vp, i32, i64, i64, vp, vp]),
    "smlu_refactor_csc": (i32, [vp, i64, vp, vp, vp]),
    "smlu_solve": (i32, [vp, vp, vp]),
    "smlu_solve_device": (i32, [vp, vp, vp]),
    "smlu_residual_device": (i32, [vp, vp, vp, vp, vp]),
    "smlu_solve_multi": (i32, [vp, i64, vp, i64, vp, i64]),
    "smlu_solve_multi_device": (i32, [vp, i64, vp, i64, vp, i64]),
    "smlu_create_i32": (i32, [i64, vp, vp, vp, ctypes.POINTER(SmluOpts), ctypes.POINTER(vp)]),
    "smlu_create_z": (i32, [i64, vp, vp, vp, ctypes.POINTER(SmluOpts), ctypes.POINTER(vp)]),
    "smlu_refactor_z": (i32, [vp, vp]),
    "smlu_refactor_z_device": (i32, [vp, vp]),
    "smlu_refactor_csc_z": (i32, [vp, i64, vp, vp, vp]),
    "smlu_lsolve": (i32, [vp, vp]),
    "smlu_rsolve": (i32, [vp, vp]),
    "smlu_chunked_setup": (i32, [vp, i64]),
    "smlu_chunked_ldiv": (i32, [vp, vp, vp]),
    "smlu_chunked_ldiv_device": (i32, [vp, vp, vp]),
    "smlu_get_sizes": (i32, [vp, i64p, i64p, i64p]),
    "smlu_get_factors": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "smlu_get_sizes_z": (i32, [vp, i64p, i64p, i64p]),
    "smlu_get_factors_z": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "smlu_destroy": (None, [vp]),
    "smlu_last_error_string": (ctypes.c_char_p, [vp]),
    "smlu_last_error_col": (i64, [vp]),
    "smlu_stat": (f64, [vp, ctypes.c_char_p]),
    "smlu_plan_create": (i32, [i64, vp, vp, ctypes.POINTER(SmluOpts), ctypes.POINTER(vp)]),
    "smlu_plan_stat": (f64, [vp, ctypes.c_char_p]),
    "smlu_plan_pattern": (i32, [vp, vp, vp, vp]),
    "smlu_plan_supernodes": (i32, [vp, vp, vp, vp]),
    "smlu_plan_fronts": (i32, [vp, vp, vp, vp]),
    "smlu_get_fronts": (i32, [vp, vp, vp, vp, vp, vp, vp]),
    "smlu_plan_destroy": (None, [vp]),
    "smlu_version": (ctypes.c_char_p, []),
    "smlu_dist_create": (i32, [i64, vp, vp, vp, ctypes.POINTER(SmluOpts), i32, i32, vp, ctypes.POINTER(vp)]),
    "smlu_rccl_unique_id": (i32, [vp]),
    "smlu_dist_create_rccl": (i32, [i64, vp, vp, vp, ctypes.POINTER(SmluOpts), i32, i32, vp, ctypes.POINTER(vp)]),
    "smlu_plan_partition": (i32, [vp, i32, vp, i64p]),
    "smlu_plan_rank_memory": (i32, [vp, i32, i32, f64p, f64p, f64p]),
    "smlu_plan_project": (f64, [vp, i32, f64, f64, f64, f64p]),
    "smlu_plan_rank_schedule": (i32, [vp, i32, i32, vp, i64, i64p, vp, vp]),
}

_lib = None


def build(force: bool = False) -> str:
    """Compile libsmlu.so in-tree (hipcc --offload-arch=gfx950)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-j8", "-C", _PKG])
    return LIB_PATH


def lib():
    """Load libsmlu.so; raise (never fall back) when it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libsmlu.so not found at {LIB_PATH}; build it with `make -C {_PKG}` "
                "(there is no CPU fallback)")
        # torch (when installed) first: its wheel carries its own HIP runtime under the same
        # soname as /opt/rocm's, and whichever is loaded first serves the process -- loaded after
        # libsmlu.so, torch finds its device layer bound to the system runtime and reports no GPU
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


# smlu_transport (include/smlu.h): callbacks of a caller-supplied transport between ranks
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, vp, i32, ctypes.POINTER(i32), ctypes.POINTER(vp),
                               ctypes.POINTER(i64), ctypes.POINTER(vp), ctypes.POINTER(i64), vp)
BCAST_FN = ctypes.CFUNCTYPE(ctypes.c_int, vp, vp, i64, i32, i32, ctypes.POINTER(i32), vp)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, vp, ctypes.POINTER(f64), i32)


class SmluTransport(ctypes.Structure):
    _fields_ = [
        ("ctx", vp),
        ("device_memory", i32),
        ("exchange", EXCHANGE_FN),
        ("bcast", BCAST_FN),
        ("allreduce_max", ALLREDUCE_FN),
    ]


def default_opts(**kw) -> SmluOpts:
    o = SmluOpts()
    lib().smlu_default_opts(ctypes.byref(o))
    for k, v in kw.items():
        if k == "grid":
            g = list(v) + [0] * (3 - len(v))
            for i in range(3):
                o.grid[i] = int(g[i])
        else:
            setattr(o, k, v)
    return o


def ptr(a):
    """Raw data pointer of a numpy array (None for None)."""
    if a is None:
        return None
    return ctypes.c_void_p(a.ctypes.data)


def order_after_caller(h, t):
    """Point the handle's device entry points at the stream that produced tensor `t` (torch's
    current stream on t's device), so the library's reads of t wait for that work
    (smlu_set_stream).  Raw pointers get the null stream.  Pair every call with
    release_caller() (try/finally): the handle never keeps a stream the caller may destroy."""
    if h is None:
        return
    s = 0
    if hasattr(t, "is_cuda") and t.is_cuda:
        import torch
        s = torch.cuda.current_stream(t.device).cuda_stream
    lib().smlu_set_stream(h, ctypes.c_void_p(s))


def release_caller(h):
    """Back to the null stream after a device call (smlu.h: smlu_set_stream lifetime)."""
    if h is not None:
        lib().smlu_set_stream(h, ctypes.c_void_p(0))


class caller_stream:
    """with caller_stream(h, t): ... -- order_after_caller on entry, release_caller on exit."""

    def __init__(self, h, t):
        self.h, self.t = h, t

    def __enter__(self):
        order_after_caller(self.h, self.t)
        return self

    def __exit__(self, *exc):
        release_caller(self.h)
        return False


def last_error(h=None) -> str:
    s = lib().smlu_last_error_string(h)
    return s.decode() if s else ""
