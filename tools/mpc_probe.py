#!/usr/bin/env python3
"""Where k_mpc_gains spends its time (measurement tool): the fused MPC gains launch timed with HIP events for
the full fixed point (434+ iterations) and one iteration, with the cfg 5 windows (L = 50) and none (L = 2).

    python tools/mpc_probe.py [lib.so ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from gymnast_optimalcontrol_amd import _lib, trajectory_tracking as tt
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    libs = sys.argv[1:] or [_lib.LIB_PATH]
    g = np.load(os.path.join(ROOT, "tests", "golden", "task2_reference_output.npz"))
    for lib in libs:
        eng = AcrobotEngine(lib_path=os.path.abspath(lib))
        xr, ur = eng.t(g["x"]), eng.t(g["u"])
        xf, uf = eng.t(tt.X_F), eng.t(tt.U_F)
        S = xr.shape[0] - 1
        for name, L, mi in (("full", 50, 1000), ("dare_only", 2, 1000), ("one_iter", 50, 1), ("one_iter_L2", 2, 1)):
            ts = []
            for r in range(30):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                K, P, it = eng.mpc_gains(xr, ur, xf, uf, tt.Q_MPC, tt.R_MPC, L=L, nwin=S, max_iter=mi)
                e1.record()
                torch.cuda.synchronize()
                if r >= 5:
                    ts.append(e0.elapsed_time(e1))
            print(f"{os.path.basename(lib):20s} {name:12s} L={L:3d} iters={int(it.item()):5d} median {np.median(ts)*1e3:8.1f} us",
                  flush=True)


if __name__ == "__main__":
    main()
