"""Dev: phase timing of the fused 64-column panel (k_panel_blk<16, 2>) at 128^3 from the kernel's own
clock marks (smlu_dev_panel_trace; workgroup 0 of every launch of one refactor): start, blocks
begin (tile loaded), blocks done, tail start, row interchanges done, diagonal-block inverses done,
off-diagonal blocks done, tail end, end.  Prints the median interval per phase.

    (library built with -DSMLU_PANEL_TRACE) SMLU_LIB=... python tools/panel_trace.py [--side 128]
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
    args = ap.parse_args()
    import torch
    import smlu
    import smlu._lib as C
    from smlu import matrices as mats
    A = mats.poisson3d(args.side)
    F = smlu.ParallelSparseLU(A, profile=False)
    torch.cuda.synchronize()
    lib = C.lib()
    fn = lib.smlu_dev_panel_trace
    fn.argtypes = [ctypes.c_longlong, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    n = 4096
    assert fn(n, None) == 0
    smlu.lu_(F, A)
    torch.cuda.synchronize()
    out = np.zeros(n * 16, np.int64)
    assert fn(0, out.ctypes.data) == 0
    t = out.reshape(n, 16)[:, :8].astype(np.float64) * 10e-3   # us
    t = t[t[:, 0] > 0]
    print(f"launches traced: {len(t)}")
    names = ["start->blocks", "blocks", "blocks->tail", "row swaps", "diag inverses", "offdiag MFMA",
             "tail->end(6)", "6->7 (rowperm, swaps, info)"]
    d = np.diff(t, axis=1)
    for k in range(7):
        col = d[:, k]
        col = col[np.isfinite(col) & (col >= 0)]
        if len(col):
            print(f"  {names[k]:30s} median {np.median(col):7.2f} us  p90 {np.percentile(col, 90):7.2f}")
    tot = t[:, 7] - t[:, 0]
    print(f"  total (mark 0 -> 7)            median {np.median(tot):7.2f} us")
    # block hand-off (shader cycles, slots 8..15): blocks 7 and 8 of launches with >= 9 blocks
    c = out.reshape(n, 16)[:, 8:].astype(np.float64)
    c = c[(c[:, 0] > 0) & (c[:, 7] > 0)]
    if len(c):
        print(f"block hand-off, shader cycles (median over {len(c)} launches):")
        for b in range(2):
            o = 4 * b
            print(f"  block {7 + b}: owner factors {np.median(c[:, o + 1] - c[:, o]):6.0f}, "
                  f"owner end -> next wave past barrier {np.median(c[:, o + 2] - c[:, o + 1]):6.0f}, "
                  f"next wave applies {np.median(c[:, o + 3] - c[:, o + 2]):6.0f}")
        print(f"  block 7 owner start -> block 8 owner start {np.median(c[:, 4] - c[:, 0]):6.0f}")
    F.close()


if __name__ == "__main__":
    main()
