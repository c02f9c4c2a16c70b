#!/usr/bin/env python3
"""Profiling driver (GPU): the general (tau1-streaming, U0Z = false) and the specialised (tau1-zero) phase kernels
of the pipelined schedule in ONE process, alternating, on the bench workload (262,144 lanes, th ~ U(+-0.5)) for a
fixed number of iterations (all lanes active: every phase launch is a full one).  Run under rocprofv3
(tools/r04_general_profile.sh) so that k_nt_phase<false, ...> and k_nt_phase<true, ...> are traced / counted on the
same box, the same buffers' sizes and the same process.

    python tools/phase_pair.py [--iters 20] [--rounds 2]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import load_refs, make_x0  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--batch", type=int, default=262144)
    a = ap.parse_args()
    import torch
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr, ur = load_refs()
    eng = AcrobotEngine()
    x0 = eng.t(make_x0(a.batch))
    kw = dict(tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20, pipeline=True, tail_lanes=0, compact=False)
    solvers = {"general": BatchedNewtonSolver(eng, xr, ur, a.batch, u0_zero=False, **kw).enable_timing(),
               "u0zero": BatchedNewtonSolver(eng, xr, ur, a.batch, **kw).enable_timing()}
    assert solvers["u0zero"].u0_zero and not solvers["general"].u0_zero
    for name, s in solvers.items():      # warm-up
        s.solve(x0, 2, sync_every=4)
        s.reset_timing()
    for r in range(a.rounds):
        for name, s in solvers.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            s.solve(x0, a.iters, sync_every=4)
            torch.cuda.synchronize()
            kt = s.kernel_times()
            ms = sum(kt[k][0] for k in ("phase_odd", "phase_even"))
            n = sum(kt[k][1] for k in ("phase_odd", "phase_even"))
            print(f"round {r} {name}: {time.perf_counter() - t0:.3f} s, phase {ms / max(n, 1):.1f} ms avg over {n}"
                  f" launches (HIP events)", flush=True)
            s.reset_timing()


if __name__ == "__main__":
    main()
