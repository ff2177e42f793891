"""The sync-free triangular sweep of the large fronts (k_tri_sweep: one launch per level and
direction, chunks of 256 rows chained by flags in ticket order) against the oracle's ldiv!
(src/SharedMemSparseLU.jl:286-342) and against the previous one-launch-per-64-column-block
schedule (SMLU_SOLVE_STEPS=1; batched right-hand sides keep it), bitwise, and the sequence that
broke the round-2 flag-chained solve: single-vector solves, then batches of every width, then
single solves again, every batch column bitwise equal to its single solve."""
import numpy as np
import pytest
import scipy.sparse as sp

import oracle as O
import smlu
from smlu import matrices as mats

from _parity import TOL, DENSE_TOL, isapprox

pytestmark = pytest.mark.gpu


def _cases():
    rng = np.random.default_rng(77)
    D = rng.random((1100, 1100)) + 1100 * np.eye(1100) * rng.random(1100)
    return {"poisson3d_28": mats.poisson3d(28),            # root separator 784 pivots, 13 blocks
            "poisson2d_300": mats.poisson2d(300),          # root separator 300 pivots, tall fronts below
            "dense_1100": sp.csc_matrix(D)}                # one front, 18 blocks, 5 chunks


@pytest.mark.parametrize("name", ["poisson3d_28", "poisson2d_300", "dense_1100"])
def test_sweep_matches_oracle_and_step_schedule(gpu, monkeypatch, name):
    import torch
    A = _cases()[name]
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A)
    assert F.stat("solve_sweeps") > 0
    b = np.random.default_rng(1).random(n)
    x = np.empty(n)
    smlu.ldiv_(x, F, b)
    ref = O.OracleLU(A, F.p, F.q)
    xo = np.empty(n)
    ref.ldiv(xo, b)
    tol = DENSE_TOL if name.startswith("dense") else TOL
    assert isapprox(x, xo, tol, tol)
    # lsolve!/rsolve! through the sweeps (single direction each) against the oracle's
    w = np.random.default_rng(2).random(n)
    wl = w.copy()
    smlu.lsolve_(F, wl)
    assert np.allclose(wl, ref.lsolve(w.copy()), rtol=1e-12, atol=1e-12 * abs(w).max())
    wu = w.copy()
    smlu.rsolve_(F, wu)
    xr = ref.rsolve(w.copy())
    assert np.linalg.norm(wu - xr) <= 1e-10 * np.linalg.norm(xr)
    # the previous per-block schedule gives the same solution to rounding
    monkeypatch.setenv("SMLU_SOLVE_STEPS", "1")
    F2 = smlu.ParallelSparseLU(A)
    monkeypatch.delenv("SMLU_SOLVE_STEPS")
    assert F2.stat("solve_sweeps") == 0
    x2 = np.empty(n)
    smlu.ldiv_(x2, F2, b)
    assert np.array_equal(x, x2)   # the same per-block arithmetic in the same order: bitwise
    assert F.stat("sweep_timeouts") == 0
    F.close()
    F2.close()


def test_single_batch_single_sequence_bitwise(gpu):
    # the order that faulted the round-2 flag-chained solve at 128^3: single, batched, single
    import torch
    A = mats.poisson3d(40)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A)
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(9)
    b = torch.from_numpy(rng.random(n)).to(dev)
    x = torch.empty_like(b)
    F.solve_device(x, b)
    x_first = x.clone()
    for k in (2, 4, 8, 16):
        B = torch.from_numpy(rng.random((k, n))).to(dev)
        X = torch.empty_like(B)
        F.solve_multi_device(X, B)
        for j in range(k):
            F.solve_device(x, B[j].contiguous())
            assert torch.equal(x, X[j]), (k, j)
    F.solve_device(x, b)
    assert torch.equal(x, x_first)
    xh = x.cpu().numpy()
    bh = b.cpu().numpy()
    assert np.abs(A @ xh - bh).max() <= 1e-12 * np.abs(bh).max()
    assert F.stat("sweep_timeouts") == 0
    F.close()


@pytest.mark.parametrize("name", ["poisson3d_28", "dense_1100"])
def test_forced_sweep_timeout_reruns_per_block(gpu, monkeypatch, name):
    """A sweep wait that gives up must never leave a wrong x: with SMLU_SWEEP_SPIN=0
    every wait reports a timeout; each solve reads the flag back, re-runs on the per-block schedule
    and returns the per-block schedule's x bitwise -- for ldiv! into a separate x, in place
    (x === b, the input kept for the re-run), and for the in-place lsolve!/rsolve!."""
    import torch
    A = _cases()[name]
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A)                        # normal spin bound
    monkeypatch.setenv("SMLU_SWEEP_SPIN", "0")
    Ft = smlu.ParallelSparseLU(A)                       # every sweep wait times out
    monkeypatch.delenv("SMLU_SWEEP_SPIN")
    assert Ft.stat("solve_sweeps") > 0
    b = np.random.default_rng(5).random(n)
    x = np.empty(n)
    smlu.ldiv_(x, F, b)
    xt = np.empty(n)
    smlu.ldiv_(xt, Ft, b)
    t1 = Ft.stat("sweep_timeouts")   # one per solve (refined solves: one per refinement solve)
    assert t1 >= 1 and Ft.stat("sweep_status") == 0
    assert np.array_equal(x, xt)
    # x === b on the device
    dev = torch.device("cuda:0")
    bd = torch.from_numpy(b).to(dev)
    Ft.solve_device(bd, bd)
    assert np.array_equal(bd.cpu().numpy(), x)
    assert Ft.stat("sweep_timeouts") > t1
    # lsolve!/rsolve! in place
    w = np.random.default_rng(6).random(n)
    wl, wlt = w.copy(), w.copy()
    smlu.lsolve_(F, wl)
    smlu.lsolve_(Ft, wlt)
    assert np.array_equal(wl, wlt)
    wu, wut = w.copy(), w.copy()
    smlu.rsolve_(F, wu)
    smlu.rsolve_(Ft, wut)
    assert np.array_equal(wu, wut)
    assert Ft.stat("sweep_timeouts") >= t1 + 3
    assert F.stat("sweep_timeouts") == 0
    F.close()
    Ft.close()

