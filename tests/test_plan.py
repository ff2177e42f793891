"""CPU tests of the host symbolic analysis (no GPU): the plan's L pattern is exactly the
structural fill of (Rs.*A)[q,q] computed independently by the oracle, for structurally
symmetric inputs; a superset for unsymmetric ones; supernode/level invariants hold."""
import os
import numpy as np
import pytest
import scipy.sparse as sp

import oracle as O
import smlu
from smlu import matrices as mats


def pattern(M):
    M = sp.csc_matrix(M, copy=True)
    M.data[:] = 1.0
    return M


def fill_pattern(A, q):
    F = O.OracleLU(A, q, q)
    return pattern(F.L), pattern(F.U)


CASES = [
    ("poisson2d_10", lambda: mats.poisson2d(10), {}),
    ("poisson2d_16_geo", lambda: mats.poisson2d(16), {"grid": (16, 16)}),
    ("poisson3d_6_geo", lambda: mats.poisson3d(6), {"grid": (6, 6, 6)}),
    ("poisson3d_9", lambda: mats.poisson3d(9), {}),
    ("poisson3d_8_natural", lambda: mats.poisson3d(8), {"ordering": "natural"}),
    ("poisson3d_8_norelax", lambda: mats.poisson3d(8), {"relax": False}),
    ("fe_20", lambda: O.test_matrix(np.random.default_rng(1), 20, 5), {}),
    ("fe_1", lambda: O.test_matrix(np.random.default_rng(1), 1, 5), {}),
    ("dense_30", lambda: sp.csc_matrix(np.random.default_rng(2).random((30, 30))), {}),
    ("dense_1", lambda: sp.csc_matrix(np.ones((1, 1))), {}),
    ("diag_7", lambda: sp.identity(7, format="csc"), {}),
    ("sym_random", lambda: sp.csc_matrix((lambda R: R + R.T + sp.identity(150))(
        sp.random(150, 150, density=0.02, random_state=3))), {}),
    ("poisson2d_20_amd", lambda: mats.poisson2d(20), {"ordering": "amd"}),
    ("poisson3d_9_amd", lambda: mats.poisson3d(9), {"ordering": "amd"}),
    ("fe_20_amd", lambda: O.test_matrix(np.random.default_rng(1), 20, 5), {"ordering": "amd"}),
    ("sym_random_amd", lambda: sp.csc_matrix((lambda R: R + R.T + sp.identity(150))(
        sp.random(150, 150, density=0.02, random_state=3))), {"ordering": "amd"}),
    ("dense_30_amd", lambda: sp.csc_matrix(np.random.default_rng(2).random((30, 30))), {"ordering": "amd"}),
    ("diag_7_amd", lambda: sp.identity(7, format="csc"), {"ordering": "amd"}),
]


@pytest.mark.parametrize("name,make,kw", CASES, ids=[c[0] for c in CASES])
def test_plan_pattern_equals_structural_fill(name, make, kw):
    A = sp.csc_matrix(make())
    P = smlu.Plan(A, **kw)
    q = P.q()
    assert np.array_equal(np.sort(q), np.arange(A.shape[0]))
    Lp = P.L_pattern()
    Lo, Uo = fill_pattern(A, q)
    assert abs(Lp - Lo).count_nonzero() == 0
    assert abs(Lp.T - Uo).count_nonzero() == 0
    assert P.stat("nnzL") == Lo.nnz


@pytest.mark.parametrize("seed", range(4))
def test_plan_pattern_superset_unsymmetric(seed):
    n = 120
    A = sp.csc_matrix(sp.random(n, n, density=0.03, random_state=seed) + sp.identity(n))
    P = smlu.Plan(A)
    q = P.q()
    Lp = P.L_pattern()
    Lo, Uo = fill_pattern(A, q)
    assert (Lo - Lo.multiply(Lp)).count_nonzero() == 0       # oracle fill contained
    assert (Uo - Uo.multiply(Lp.T)).count_nonzero() == 0


def test_supernode_and_level_invariants():
    A = mats.poisson3d(12)
    P = smlu.Plan(A)
    first, parent, level = P.supernodes()
    ns = len(parent)
    assert first[0] == 0 and first[-1] == A.shape[0] and np.all(np.diff(first) > 0)
    for s in range(ns):
        if parent[s] >= 0:
            assert parent[s] > s
            assert level[parent[s]] > level[s]
    assert P.stat("nlevels") == level.max() + 1


def test_graph_nd_beats_natural_fill():
    A = mats.poisson3d(16)
    nd = smlu.Plan(A).stat("nnzL")
    nat = smlu.Plan(A, ordering="natural").stat("nnzL")
    geo = smlu.Plan(A, grid=(16, 16, 16)).stat("nnzL")
    assert nd < nat and geo < nat


def test_geometric_needs_matching_grid():
    with pytest.raises(RuntimeError):
        smlu.Plan(mats.poisson2d(8), ordering="geometric", grid=(7, 8))


def test_plan_rejects_bad_pattern():
    A = sp.csc_matrix(np.eye(3))
    A.indices = np.array([0, 5, 2], dtype=A.indices.dtype)   # row out of range
    with pytest.raises(RuntimeError):
        smlu.Plan(A)


def test_flop_and_update_counts_match_oracle():
    A = mats.poisson2d(12)
    P = smlu.Plan(A, relax=False)
    q = P.q()
    Lo, Uo = fill_pattern(A, q)
    # upd = sum_k |L_k| * |U_k| over strictly off-diagonal counts
    lk = np.diff(Lo.indptr) - 1
    uk = np.diff(sp.csr_matrix(Uo).indptr) - 1
    assert P.stat("upd") == float(np.sum(lk * uk))


@pytest.mark.parametrize("make", [lambda: mats.poisson2d(60), lambda: mats.poisson3d(14),
                                  lambda: sp.csc_matrix((lambda R: R + R.T + sp.identity(800))(
                                      sp.random(800, 800, density=0.004, random_state=5)))],
                         ids=["poisson2d_60", "poisson3d_14", "sym_random_800"])
def test_amd_fill_close_to_minimum_degree(make):
    """SMLU_ORDER_AMD (csrc/amd.cpp) against an independent minimum-degree code: SuperLU's
    MMD on A+A' (scipy), no pivoting, symmetric mode.  nnz(L+U) of our unrelaxed symbolic
    factor within 15 %, and far below the natural order's."""
    import scipy.sparse.linalg as spla
    A = sp.csc_matrix(make())
    n = A.shape[0]
    amd = smlu.Plan(A, ordering="amd", relax=False)
    nnz_amd = 2 * amd.stat("nnzL") - n
    lu = spla.splu(A, permc_spec="MMD_AT_PLUS_A", diag_pivot_thresh=0.0,
                   options=dict(SymmetricMode=True))
    nnz_mmd = lu.L.nnz + lu.U.nnz - n
    nat = smlu.Plan(A, ordering="natural", relax=False)
    assert nnz_amd <= 1.15 * nnz_mmd, (nnz_amd, nnz_mmd)
    assert nnz_amd < 2 * nat.stat("nnzL") - n


def test_bench_ordering_compare():
    """bench.py's config.ordering_compare: ND and AMD statistics from the host analysis, the
    numbers DESIGN.md §1 quotes (ND fills less than AMD on 3D grids)."""
    import importlib
    import sys as _sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in _sys.path:
        _sys.path.insert(0, root)
    bench = importlib.import_module("bench")
    out = bench.ordering_compare(14)
    c3, c2 = out["c3_poisson3d_14"], out["c2_poisson2d_512"]
    for row in (c3, c2):
        for o in ("nd", "amd"):
            assert row[o]["nnzLU"] > 0 and row[o]["upd"] > 0
    assert c3["nd"]["upd"] < c3["amd"]["upd"]


_PLAN_HASH = """
import hashlib, sys
sys.path.insert(0, %r)
import numpy as np
import smlu
from smlu import matrices as mats
P = smlu.Plan(mats.poisson3d(64))
first, parent, rowptr, rows, p0 = P.fronts()
h = hashlib.sha256()
for a in (first, parent, rowptr, rows, p0):
    h.update(np.ascontiguousarray(a, np.int64).tobytes())
print(h.hexdigest())
"""


def test_plan_independent_of_thread_count():
    """The threaded analysis (nested-dissection halves on their own threads above 200k vertices,
    row structures by tree height, the A map's parallel sort) gives the same plan on 1 thread as
    on the default count: 64^3 forks at the top bisection."""
    import subprocess
    import sys
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sharedmemsparselu.jl_amd")
    out = []
    for threads in ("1", None):
        env = dict(os.environ)
        env.pop("OMP_NUM_THREADS", None)
        if threads:
            env["OMP_NUM_THREADS"] = threads
        r = subprocess.run([sys.executable, "-c", _PLAN_HASH % pkg], env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr
        out.append(r.stdout.strip())
    assert out[0] == out[1]
