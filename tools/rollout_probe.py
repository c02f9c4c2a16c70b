#!/usr/bin/env python3
"""Time the cfg 5 closed-loop rollout (gym_track_rollout_ex, 8,192 lanes x 500 steps) for library variants
(measurement tool): median of 30 launches timed with HIP events on the engine's stream.

    python tools/rollout_probe.py lib_a.so lib_b.so ...
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    g = np.load(os.path.join(ROOT, "tests", "golden", "task2_reference_output.npz"))
    rng = np.random.default_rng(0)
    B = 8192
    x0 = g["x"][0][None, :] + rng.normal(0, 0.05, (B, 4))
    K = rng.normal(0, 1.0, (g["u"].shape[0], 2, 4)) * 0.1
    for lib in sys.argv[1:]:
        eng = AcrobotEngine(lib_path=os.path.abspath(lib))
        ts = []   # the engine launches on torch's current stream (engine.stream), where the events are recorded
        xd, xf, uf, Kd = eng.t(x0), eng.t(g["x"]), eng.t(g["u"]), eng.t(K)
        for r in range(33):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            x, u = eng.track_rollout(xd, xf, uf, Kd)
            e1.record()
            torch.cuda.synchronize()
            if r >= 3:
                ts.append(e0.elapsed_time(e1))
        print(f"{os.path.basename(lib)}: rollout {np.median(ts) * 1e3:.1f} us (min {min(ts) * 1e3:.1f}), "
              f"x[0,-1] {x[0, -1].cpu().numpy()}", flush=True)


if __name__ == "__main__":
    main()
