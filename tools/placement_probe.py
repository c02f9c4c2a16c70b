#!/usr/bin/env python3
"""Does a short run tell a slow buffer placement from a fast one?  (measurement tool)

    python tools/placement_probe.py --sets 5 --out gpurun_out/r05/placement/probe.json

The headline phase kernel's time depends on where its stream buffers land (one box: 1.92-2.06 ms per launch for the
same kernel on different allocations; profiles/r05/place*/).  This allocates --sets solvers of the headline workload
(each its own x / u / K1 / cs buffers, all alive at once), and for each records the phase kernel's average over a
short probe (the first --probe-iters iterations of a solve) and over a full solve, to see whether the probe predicts
the solve.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=5)
    ap.add_argument("--probe-iters", type=int, default=8)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import torch
    import bench
    from gymnast_optimalcontrol_amd import distributed as gd
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    torch.cuda.set_device(0)
    x_ref, u_ref = bench.load_refs()
    eng = AcrobotEngine()
    ns = argparse.Namespace(spread=0.5, schedule="auto", chunk=128, split_waves="on", tail_lanes=None, compact="auto",
                            max_iters=5000, sync_every=4)
    legs = [bench.NewtonLeg(ns, gd, eng, x_ref, u_ref, 262144, True) for _ in range(a.sets)]
    out = []

    def phase_avg(sv):
        kt = sv.kernel_times()
        ms = sum(kt[k][0] for k in ("phase_odd", "phase_even"))
        n = sum(kt[k][1] for k in ("phase_odd", "phase_even"))
        return ms / max(n, 1)

    for rnd in range(2):
        for i, leg in enumerate(legs):
            sv = leg.solver
            sv.reset_timing()
            sv.solve(leg.x0_dev, a.probe_iters, sync_every=4)       # the probe: the first iterations only
            torch.cuda.synchronize()
            sv.collect_timing()
            probe = phase_avg(sv)
            sv.reset_timing()
            t0 = time.perf_counter()
            r = sv.solve(leg.x0_dev, 5000, sync_every=4)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            full = phase_avg(sv)
            rec = {"round": rnd, "set": i, "x0": hex(sv.x[0].data_ptr()), "K1": hex(sv.K1.data_ptr()),
                   "probe_phase_ms": probe, "solve_phase_ms": full, "it_per_s": r.lane_iterations / dt}
            out.append(rec)
            print(json.dumps(rec), flush=True)
            r = None
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
