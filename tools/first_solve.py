#!/usr/bin/env python3
"""Where does a solver's first solve spend its extra time?  (measurement tool; the bench line's `setup` record)

    python tools/first_solve.py --out gpurun_out/r06/first/first.json

One process, the headline workload (262,144 lanes): A = a cold solver (the process's first GPU work beyond the
engine) and its first solve (placement selection inside it); B = a second solver after PlacementPool.clear() (warm
process, selection again); C = a third solver of the same shape, which takes B's set from the pool (no selection),
then three more solves on C.  For each solve: wall time, iterations, and the host timeline of its statistics reads
(every 4 iterations), so the probe blocks, the state copies and any one-time cost show where they fall.
"""
import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=262144)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import torch
    import bench
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver, PlacementPool
    torch.cuda.set_device(0)
    x_ref, u_ref = bench.load_refs()
    eng = AcrobotEngine()
    x0 = eng.t(bench.make_x0(a.lanes))
    torch.cuda.synchronize()
    recs = []

    def build(tag):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s = BatchedNewtonSolver(eng, x_ref, u_ref, a.lanes, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"build": tag, "setup_s": dt}), flush=True)
        return s, dt

    def solve(tag, s, setup):
        s.timeline = []
        t0 = time.perf_counter()
        r = s.solve(x0, 5000, sync_every=4)
        dt = time.perf_counter() - t0
        tl = [(k, n, round(t - t0, 4)) for k, n, t in s.timeline]
        rec = {"solve": tag, "setup_s": setup, "seconds": dt, "solver_seconds": r.seconds, "iterations": r.iterations,
               "lane_iterations": r.lane_iterations, "placement": s.placement,
               "t_at_iteration": {str(k): t for k, _, t in tl if k in (4, 12, 24, 48, 96, 100, 200, 300, 400)},
               "timeline": tl}
        print(json.dumps({k: v for k, v in rec.items() if k != "timeline"}), flush=True)
        recs.append(rec)
        return r

    sa, ta = build("A")
    solve("A_first", sa, ta)
    solve("A_second", sa, 0.0)
    del sa
    gc.collect()
    PlacementPool.clear()
    sb, tb = build("B")
    solve("B_first", sb, tb)
    del sb
    gc.collect()
    sc, tc = build("C_pooled")
    solve("C_first", sc, tc)
    for i in range(3):
        solve(f"C_{i + 2}", sc, 0.0)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(recs, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
