"""CPU tests of the drop-in boundary: libsmlu.so loads, exports every function declared in
include/smlu.h, validates arguments, and fails loudly (no CPU fallback) without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest
import scipy.sparse as sp

import smlu
from smlu import _lib as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "smlu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(smlu_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def test_header_declares_expected_surface():
    names = header_functions()
    for n in ("smlu_create", "smlu_refactor", "smlu_solve", "smlu_lsolve", "smlu_rsolve",
              "smlu_get_factors", "smlu_destroy", "smlu_create_with_pivots"):
        assert n in names


def test_library_exports_every_header_symbol():
    L = smlu.lib()
    for name in header_functions():
        assert hasattr(L, name), f"{name} declared in smlu.h but not exported"
        assert name in C.SIGNATURES, f"{name} has no ctypes signature"


def test_nm_exports_are_c_abi():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", C.LIB_PATH], capture_output=True, text=True).stdout
    for name in header_functions():
        assert re.search(rf"\bT {name}$", out, flags=re.M), f"{name} not an unmangled export"
    # and nothing else: the library is built with -fvisibility=hidden, so the internal C++
    # functions (launch wrappers, plan, schedule) stay inside it
    exported = set(re.findall(r"^\S+ T (\S+)$", out, flags=re.M))
    assert exported == set(header_functions()), sorted(exported ^ set(header_functions()))


def test_version_and_defaults():
    assert b"gfx950" in smlu.lib().smlu_version()
    o = C.default_opts()
    assert o.index_base == 1 and o.chunk_size == 8 and o.scale == 1
    assert abs(o.pivot_tol - 0.1) < 1e-15


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU failure mode")
def test_create_fails_loudly_without_gpu():
    A = sp.csc_matrix(np.eye(4))
    with pytest.raises(smlu.SmluError, match="no HIP device"):
        smlu.ParallelSparseLU(A)


def test_create_argument_validation():
    L = smlu.lib()
    h = ctypes.c_void_p()
    rc = L.smlu_create(0, None, None, None, None, ctypes.byref(h))
    assert rc == C.SMLU_ERR_ARG
    assert C.last_error(None)


def test_not_square_is_dimension_mismatch():
    with pytest.raises(smlu.DimensionMismatch):
        smlu.ParallelSparseLU(sp.csc_matrix(np.ones((3, 4))))


def test_null_handle_calls_are_safe():
    L = smlu.lib()
    assert L.smlu_refactor(None, None) == C.SMLU_ERR_ARG
    assert L.smlu_solve(None, None, None) == C.SMLU_ERR_ARG
    assert L.smlu_chunked_setup(None, 8) == C.SMLU_ERR_ARG
    assert L.smlu_chunked_ldiv(None, None, None) == C.SMLU_ERR_ARG
    assert L.smlu_chunked_ldiv_device(None, None, None) == C.SMLU_ERR_ARG
    assert L.smlu_last_error_col(None) == -1
    L.smlu_destroy(None)
    assert np.isnan(L.smlu_stat(None, b"n"))


def test_plan_one_based_input():
    """Julia passes 1-based colptr/rowval (index_base = 1, the default)."""
    A = sp.csc_matrix(np.array([[4.0, 1, 0], [1, 4, 1], [0, 1, 4]]))
    cp = (A.indptr + 1).astype(np.int64)
    ri = (A.indices + 1).astype(np.int64)
    o = C.default_opts()
    h = ctypes.c_void_p()
    rc = smlu.lib().smlu_plan_create(3, C.ptr(cp), C.ptr(ri), ctypes.byref(o), ctypes.byref(h))
    assert rc == 0
    assert smlu.lib().smlu_plan_stat(h, b"nnzL") == 5.0  # tridiagonal: no fill
    smlu.lib().smlu_plan_destroy(h)


def test_allocate_shared_stub():
    z = smlu.allocate_shared(np.float64, 3, 2)
    assert z.shape == (3, 2) and not z.any()
