#!/usr/bin/env python3
"""Active lanes against iterations and time over one stress-workload solve (diagnostic).

    python tools/stress_timeline.py [--tail-lanes N] [--batch B] [--spread 1.5]

Prints the active-lane count and the elapsed time at every host synchronisation (every 4 iterations on the lock-step
schedules; after each straggler-tail launch), condensed to a few dozen rows."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tail-lanes", type=int, default=None)
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--spread", type=float, default=1.5)
    a = ap.parse_args()
    import torch
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    x_ref, u_ref = load_refs()
    eng = AcrobotEngine()
    s = BatchedNewtonSolver(eng, x_ref, u_ref, a.batch, tol=1e-4, gamma_0=0.1, tail_lanes=a.tail_lanes)
    x0 = eng.t(make_x0(a.batch, spread=a.spread))
    s.solve(x0, 5000, sync_every=4)                       # warm-up
    s.timeline = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = s.solve(x0, 5000, sync_every=4)
    t1 = time.perf_counter()
    tl = s.timeline
    print(f"schedule {r.schedule}, tail threshold {s.tail_lanes}, solve {t1 - t0:.3f} s, iterations {r.iterations}, "
          f"tail lane-iterations {r.tail_lane_iterations} of {r.lane_iterations}")
    marks = {0}
    for i in range(1, len(tl)):
        if tl[i][1] != tl[i - 1][1] and (len(marks) < 60 or tl[i][1] < 64):
            marks.add(i)
    step = max(len(tl) // 40, 1)
    marks |= set(range(0, len(tl), step)) | {len(tl) - 1}
    for i in sorted(marks):
        k, act, t = tl[i]
        print(f"  iter {k:5d}  active {act:7d}  t {t - t0:7.3f} s")


if __name__ == "__main__":
    main()
