#!/usr/bin/env python3
"""Bitwise comparison of the cfg 5 MPC outputs of library variants (measurement tool): the fused gains
(gym_mpc_gains: gains, P_inf, fixed-point iterations) and the closed-loop rollout of 8,192 disturbed starts,
each library's against the first one's.

    GYM_ALLOW_FOREIGN_BUILD=1 python tools/mpc_libs_compare.py lib_a.so lib_b.so ...
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from gymnast_optimalcontrol_amd import trajectory_tracking as tt
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    g = np.load(os.path.join(ROOT, "tests", "golden", "task2_reference_output.npz"))
    rng = np.random.default_rng(0)
    B = 8192
    x0 = g["x"][0][None, :] + rng.normal(0, 0.05, (B, 4))
    ref = None
    for lib in sys.argv[1:]:
        eng = AcrobotEngine(lib_path=os.path.abspath(lib))
        xr, ur = eng.t(g["x"]), eng.t(g["u"])
        xf, uf = eng.t(tt.X_F), eng.t(tt.U_F)
        S = xr.shape[0] - 1
        K, P, it = eng.mpc_gains(xr, ur, xf, uf, tt.Q_MPC, tt.R_MPC, L=50, nwin=S, max_iter=1000)
        x, u = eng.track_rollout(eng.t(x0), xr, ur, K)
        torch.cuda.synchronize()
        out = {"K": K.cpu().numpy(), "P": P.cpu().numpy(), "it": it.cpu().numpy(), "x": x.cpu().numpy(),
               "u": u.cpu().numpy()}
        if ref is None:
            ref = out
            print(f"{os.path.basename(lib)}: reference (fixed-point iterations {int(out['it'])})", flush=True)
            continue
        same = {k: bool(np.array_equal(out[k], ref[k], equal_nan=True)) for k in out}
        print(f"{os.path.basename(lib)}: bitwise equal {same}", flush=True)
        if not all(same.values()):
            sys.exit(1)


if __name__ == "__main__":
    main()
