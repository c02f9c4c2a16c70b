#!/usr/bin/env python3
"""Where the two-wavefront persistent kernel (k_nt_run2) spends its cycles (diagnostic tool).

    python tools/run2_trace.py build_ab/run2_trace.so [--batch 4096] [--iters 40]

The library is built with -DGYM_RUN2_TRACE (_build.build(defines=["GYM_RUN2_TRACE"], out=...)).  Prints, per
wavefront role (main / helper), the mean cycles per iteration in the sweep, the trial, the post-trial part and
waiting at the chunk barriers (s_memtime cycles, workgroups averaged)."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    os.environ["GYM_ALLOW_FOREIGN_BUILD"] = "1"     # a define-variant of this tree (its build id differs)
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--single", action="store_true", help="the single-wavefront kernel k_nt_run (main role only)")
    a = ap.parse_args()
    import torch
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    eng = AcrobotEngine(lib_path=os.path.abspath(a.lib))
    eng.lib.gym_debug_run2_trace.argtypes = [C.c_void_p, C.c_int]
    x_ref, u_ref = load_refs()
    s = BatchedNewtonSolver(eng, x_ref, u_ref, a.batch, tol=1e-4, gamma_0=0.1, persistent=True, chunk=0,
                            split_waves=not a.single)
    x0 = make_x0(a.batch)
    s.solve(x0, a.iters)                          # warm-up
    buf = np.zeros((8192, 2, 6), np.uint64)
    eng.lib.gym_debug_run2_trace(buf.ctypes.data, 1)
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True); t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    r = s.solve(x0, a.iters)
    t1.record(); torch.cuda.synchronize()
    eng.lib.gym_debug_run2_trace(buf.ctypes.data, 0)
    nb = (a.batch + 63) // 64
    tr = buf[:nb].astype(np.float64)
    it = tr[:, 0, 3]
    print(f"B={a.batch} iters={a.iters} solve {t0.elapsed_time(t1):.2f} ms, mean iterations per workgroup {it.mean():.1f}")
    for role, name in ((0, "main"), (1, "helper")):
        per = tr[:, role, [0, 1, 2, 4, 5]] / np.maximum(tr[:, role, 3:4], 1)
        print(f"  {name:6s} cycles/iteration: sweep {per[:, 0].mean():9.0f} (barrier wait {per[:, 3].mean():8.0f})  "
              f"trial {per[:, 1].mean():9.0f} (barrier wait {per[:, 4].mean():8.0f})  post {per[:, 2].mean():8.0f}")
    T = x_ref.shape[0] - 1
    print(f"  per stage: sweep {tr[:, 0, 0].sum() / tr[:, 0, 3].sum() / T:.0f}  trial {tr[:, 0, 1].sum() / tr[:, 0, 3].sum() / T:.0f} cycles")


if __name__ == "__main__":
    main()
