"""Device entry points against the caller's stream (smlu_set_stream, include/smlu.h): values and
right-hand sides produced by kernels still queued on a torch side stream -- behind a long sleep
kernel -- are read only after that work, with no host synchronisation by the caller; and the
status words the library reads back (pivot status, dominance, sweep timeouts) stay right across
many refactor / solve rounds interleaved with torch work on another stream (the in-place update
pattern of tools/c5_steady.py)."""
import numpy as np
import pytest
import scipy.sparse as sp

import smlu
from smlu import matrices as mats

pytestmark = pytest.mark.gpu


def _residual(A, x, b):
    return float(np.abs(A @ x - b).max() / np.abs(b).max())


def test_inputs_from_busy_side_stream(gpu):
    import torch
    A = mats.poisson3d(24)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A, device=0)
    dev = torch.device("cuda", 0)
    dpos = torch.from_numpy(mats.diag_positions(A)).to(dev)
    base = torch.from_numpy(np.ascontiguousarray(A.data)).to(dev)
    bh = np.random.default_rng(3).random(n)
    torch.cuda.synchronize()
    s = torch.cuda.Stream(device=dev)
    for r in range(3):
        with torch.cuda.stream(s):
            torch.cuda._sleep(20_000_000)            # keep the stream busy for milliseconds
            v = base.clone()
            v[dpos] += 1.0 + r
            b = torch.from_numpy(bh).to(dev, non_blocking=False) * (r + 1)
            x = torch.empty_like(b)
            F.refactor_device(v)
            F.solve_device(x, b)
            xh = x.cpu().numpy()
        torch.cuda.synchronize()
        Al = A.copy()
        Al.data = v.cpu().numpy()
        assert _residual(Al, xh, bh * (r + 1)) < 1e-12, r
    F.close()


def test_status_reads_across_interleaved_updates(gpu):
    import torch
    A = mats.poisson3d(40)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A, device=0)
    dev = torch.device("cuda", 0)
    dpos = torch.from_numpy(mats.diag_positions(A)).to(dev)
    base = torch.from_numpy(np.ascontiguousarray(A.data)).to(dev)
    vals = torch.empty_like(base)
    g = torch.Generator(device=dev)
    b = torch.from_numpy(np.random.default_rng(5).random(n)).to(dev)
    x = torch.empty_like(b)
    for r in range(12):
        g.manual_seed(47 + r)
        vals.copy_(base)
        vals[dpos] += torch.rand(dpos.numel(), generator=g, device=dev, dtype=torch.float64)
        F.refactor_device(vals)
        assert F.stat("dominant") == 1.0 and F.stat("weak") == 0.0 and F.stat("pivmode") == 0.0, r
        F.solve_device(x, b)
    assert F.stat("repivots") == 0.0
    assert F.stat("sweep_timeouts") == 0.0
    Al = A.copy()
    Al.data = vals.cpu().numpy()
    assert _residual(Al, x.cpu().numpy(), b.cpu().numpy()) < 1e-12
    F.close()
