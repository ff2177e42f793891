"""Dev: timing structure of the root-front sync-free sweep (k_tri_sweep) at 128^3 from the kernel's
own clock marks (smlu_dev_sweep_trace): per work item (chunk of kSweepWK blocks) and wave, the 100 MHz
real-time clock at start / external blocks applied / before and after the substitution / published /
end.  Prints the per-block chain intervals and the cross-chunk hand-off gaps.

    (library built with -DSMLU_SWEEP_TRACE) python tools/sweep_trace.py [--side 128] [--wk 4]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sharedmemsparselu.jl_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=128)
    ap.add_argument("--wk", type=int, default=4)
    ap.add_argument("--nwg", type=int, default=72, help="grid of the traced launch (72: the 128^3 root front)")
    args = ap.parse_args()
    import torch
    import smlu
    import smlu._lib as C
    from smlu import matrices as mats
    A = mats.poisson3d(args.side)
    n = A.shape[0]
    F = smlu.ParallelSparseLU(A, profile=False)
    dev = torch.device("cuda:0")
    b = torch.from_numpy(np.random.default_rng(3).random(n)).to(dev)
    x = torch.empty_like(b)
    F.solve_device(x, b)
    torch.cuda.synchronize()
    lib = C.lib()
    fn = lib.smlu_dev_sweep_trace
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong]
    fn.restype = ctypes.c_int
    # root front: ns = n^(2/3)-ish; forward items = ceil(M / (64 wk)), backward ceil(nblk / wk)
    nwg = args.nwg
    for upper in (0, 1):
        items = nwg
        nrec = items * args.wk
        assert fn(items, upper, None, nrec) == 0
        F.solve_device(x, b)
        torch.cuda.synchronize()
        out = np.zeros(nrec * 8, np.int64)
        assert fn(0, 0, out.ctypes.data, nrec) == 0
        t = out.reshape(items, args.wk, 8).astype(np.float64) * 10e-3   # us
        t0 = t[:, :, 0][t[:, :, 0] > 0].min()
        t = np.where(t > 0, t - t0, np.nan)
        name = "backward" if upper else "forward"
        solved = t[:, :, 3].reshape(-1)
        ok = ~np.isnan(solved)
        print(f"{name}: items {items}, end {np.nanmax(t[:, :, 5]):.1f} us, blocks solved {ok.sum()}")
        sub = (t[:, :, 3] - t[:, :, 2]).reshape(-1)
        print(f"  substitution per block: median {np.nanmedian(sub):.2f} us, max {np.nanmax(sub):.2f}")
        intra = np.diff(t[:, :, 3], axis=1).reshape(-1)
        print(f"  solve-to-solve inside a chunk: median {np.nanmedian(intra):.2f} us")
        cross = t[1:, 0, 3] - t[:-1, -1, 3]
        print(f"  last block of chunk q-1 -> first block of chunk q: median {np.nanmedian(cross):.2f} us")
        extd = t[1:, 0, 1] - t[:-1, -1, 4]
        print(f"  published (q-1) -> externals applied (q, wave 0): median {np.nanmedian(extd):.2f} us")
        start = t[:, 0, 0]
        print(f"  item start spread: {np.nanmin(start):.1f} .. {np.nanmax(start):.1f} us")
        for q in (items // 2, items // 2 + 1):
            for w in range(args.wk):
                print(f"   q={q:3d} wave {w}: " + " ".join(f"{v:8.2f}" for v in t[q, w, :6]))
        for q in list(range(0, items, max(1, items // 8))) + [items - 1]:
            print(f"   q={q:3d} start {t[q,0,0]:8.1f} ext_done {np.nanmax(t[q,:,1]):8.1f} "
                  f"solved {' '.join(f'{v:8.1f}' for v in t[q, :, 3])} end {np.nanmax(t[q,:,5]):8.1f}")
    F.close()


if __name__ == "__main__":
    main()
