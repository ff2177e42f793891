"""Dev: the shader clock the 128x128 fp64 MFMA tile (k_gemm128_mfma3) actually runs at during 128^3
refactors, from the workgroups' own counters (smlu_dev_gemm_clock: sum of delta s_memtime over sum of
delta s_memrealtime x 100 MHz, per form: F22 = EB tile, trailing = the k = 384 / in-block tile).
The nominal fp64 matrix peak (78.6 TFLOP/s) assumes 2.4 GHz; the clock-corrected peak is
78.6 x f / 2400 MHz.

    (library built with -DSMLU_CLOCK_PROBE, see tools/gemm_clock.sh)
    SMLU_LIB=.../libsmlu_clock.so python tools/gemm_clock.py [--side 128] [--reps 3]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sharedmemsparselu.jl_amd"))

PEAK_TF = 78.6
NOMINAL_MHZ = 2400.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import smlu
    import smlu._lib as C
    from smlu import matrices as mats
    A = mats.poisson3d(args.side)
    F = smlu.ParallelSparseLU(A, profile=False)
    smlu.lu_(F, A)   # warm: graph captured
    torch.cuda.synchronize()
    fn = C.lib().smlu_dev_gemm_clock
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    assert fn(1, None) == 0
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(args.reps):
        smlu.lu_(F, A)
    ev1.record()
    torch.cuda.synchronize()
    out = np.zeros(8, np.uint64)
    assert fn(0, out.ctypes.data) == 0
    res = {"side": args.side, "reps": args.reps, "refactor_ms": ev0.elapsed_time(ev1) / args.reps}
    for form, name in ((0, "f22"), (1, "trailing_inblock")):
        cyc, real, wgs = (float(out[4 * form + i]) for i in range(3))
        if wgs == 0:
            continue
        mhz = cyc / real * 100.0
        res[name] = {"workgroups": int(wgs), "clock_mhz": round(mhz, 1),
                     "tile_us_avg": round(real / wgs / 100.0, 2),
                     "clock_corrected_peak_tflops": round(PEAK_TF * mhz / NOMINAL_MHZ, 2)}
    print(json.dumps(res))
    F.close()


if __name__ == "__main__":
    main()
