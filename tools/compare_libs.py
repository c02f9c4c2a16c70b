#!/usr/bin/env python3
"""Bitwise comparison of two builds of the HIP library on the same solver workload (diagnostic tool).

    python tools/compare_libs.py lib_a.so lib_b.so [--batch 262144] [--iters 3] [--schedule serial]

Runs ``--iters`` Newton iterations with each library on identical inputs and reports, for every
solver buffer, the lanes whose contents differ (count, first lanes, wave ids mod 16, first stage).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(lib, a, x0):
    import torch
    from bench import load_refs
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    x_ref, u_ref = load_refs()
    eng = AcrobotEngine(lib_path=os.path.abspath(lib))
    s = BatchedNewtonSolver(eng, x_ref, u_ref, a.batch, tol=1e-4, gamma_0=0.1,
                            pipeline={"serial": False, "pipelined": True, "persistent": False}[a.schedule],
                            persistent=a.schedule == "persistent")
    s.max_iters = a.iters
    s.init(x0)
    for _ in range(a.iters):
        s.iteration()
    torch.cuda.synchronize()
    return {"x0": s.x[0].cpu().numpy(), "x1": s.x[1].cpu().numpy(), "u0": s.u[0].cpu().numpy(),
            "u1": s.u[1].cpu().numpy(), "K1": s.K1.cpu().numpy(), "cs": s.cs.cpu().numpy(),
            "cost": s.cost.cpu().numpy(), "dJ": s.dJ.cpu().numpy(), "smax": s.smax.cpu().numpy()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib_a")
    ap.add_argument("lib_b")
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--schedule", choices=("serial", "pipelined", "persistent"), default="serial")
    a = ap.parse_args()
    from bench import make_x0
    x0 = make_x0(a.batch)
    A, B = run(a.lib_a, a, x0), run(a.lib_b, a, x0)
    for k in A:
        va, vb = A[k], B[k]
        # lane axis: the Bp axis (shape (..., Bp, W) for streams, (Bp,) for per-lane arrays)
        if va.ndim == 1:
            diff = ~((va == vb) | (np.isnan(va) & np.isnan(vb)))
            lanes = np.nonzero(diff)[0]
            first_stage = None
        else:
            d = ~((va == vb) | (np.isnan(va) & np.isnan(vb)))       # (L, P, Bp, W)
            per_lane = d.any(axis=(1, 3))                            # (L, Bp)
            lanes = np.nonzero(per_lane.any(axis=0))[0]
            first_stage = int(np.nonzero(per_lane.any(axis=1))[0][0]) if len(lanes) else None
        print(f"{k:5s}: {len(lanes):7d} lanes differ; first {lanes[:8].tolist()}; "
              f"waves mod 16 {sorted(set((lanes // 64 % 16).tolist()))[:16]}; first stage {first_stage}", flush=True)


if __name__ == "__main__":
    main()
