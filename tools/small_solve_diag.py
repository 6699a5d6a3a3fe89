#!/usr/bin/env python3
"""Phase times of one cycle of the one-workgroup small solve
(pinc_hip_mg_solve_small) from a diagnostic build:

    PINC_LIBDIR=pinc_amd/lib_sd PINC_HIP_DEFINES="-DPINC_SMALL_DIAG=1" python -m pinc_amd.build
    PINC_LIBDIR=pinc_amd/lib_sd python tools/small_solve_diag.py --size 128 --spectral 1

The kernel stamps s_memrealtime (100 MHz) at the phase boundaries of its
first cycle into out[2..10]; the launch itself is timed with HIP events.
"""
import argparse
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--spectral", type=int, default=1)
    ap.add_argument("--pre", type=int, default=4)
    ap.add_argument("--post", type=int, default=4)
    ap.add_argument("--cycles", type=int, default=1)
    a = ap.parse_args()
    import torch
    from pinc_amd import _lib
    import test_gpu_kernels as tk
    h = _lib.HIP
    vp = C.c_void_p
    h.pinc_hip_mg_solve_small.argtypes = [vp, vp, vp, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, vp,
                                          vp, vp]
    n = a.size
    lv = tk._small_levels(n, n)
    g = np.random.default_rng(5)
    r = g.standard_normal(n * n)
    r -= r.mean()
    rho = torch.from_numpy(r).cuda()
    basis = torch.from_numpy(tk._fourier_basis(n // 2)).cuda() if a.spectral else None
    names = ["pre-smooth", "residual out", "restrict", "coarse solve", "prolong", "reload", "post-smooth",
             "norm"]
    for rep in range(5):
        phi = torch.zeros(n * n, dtype=torch.float64, device="cuda")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = tk._small_solve(h, phi, rho, lv, a.pre, a.post, 10, a.cycles, basis)
        e1.record()
        torch.cuda.synchronize()
        t = out[2:11]
        d = np.diff(t) * 10e-3  # 100 MHz ticks -> us
        print(f"rep {rep}: launch {e0.elapsed_time(e1) * 1e3:.1f} us, cycle {(t[-1] - t[0]) * 10e-3:.1f} us: " +
              ", ".join(f"{k} {v:.1f}" for k, v in zip(names, d)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
