#!/usr/bin/env python3
"""Same-process A/B of the post-trial candidate scratch (ABI 13, measurement tool): bench.py's stress workload
(262,144 lanes, th ~ U(+-1.5), the automatic schedule) solved alternately by a solver that re-runs every accepted
Armijo candidate (cand_slots=0) and by the default one (lane-pair candidates recorded in scratch, the accepted one
copied), on one box and the same inputs; wall time per solve, the post-trial kernels' HIP-event times, and a
bitwise comparison of the two solves' outcomes.

    python tools/cand_ab.py [--rounds 3] [--lanes 262144]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--lanes", type=int, default=262144)
    ap.add_argument("--max-iters", type=int, default=5000)
    a = ap.parse_args()
    import torch
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr, ur = load_refs()
    x0 = make_x0(a.lanes, spread=1.5)
    eng = AcrobotEngine()
    kw = dict(tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20)
    solvers = {"rerun": BatchedNewtonSolver(eng, xr, ur, a.lanes, cand_slots=0, **kw).enable_timing(),
               "scratch": BatchedNewtonSolver(eng, xr, ur, a.lanes, **kw).enable_timing()}
    res = {}
    times = {k: [] for k in solvers}
    for rnd in range(a.rounds + 1):                       # round 0: warm-up
        for name, s in solvers.items():
            s.reset_timing()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = s.solve(x0, a.max_iters, sync_every=4)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            s.collect_timing()
            kt = s.kernel_times()
            its = int(r.n_iter.sum().item())
            if rnd > 0:
                times[name].append(dt)
            print(f"round {rnd} {name:8s} {dt:.3f} s  {its / dt / 1e6:.2f} M it/s  candidates "
                  f"{kt['candidates'][0]:.1f} ms / {kt['candidates'][1]}  retry {kt['retry'][0]:.1f} ms / "
                  f"{kt['retry'][1]}  tail {kt['tail'][0]:.1f} ms  (sampled post-trial pairs)", flush=True)
            res[name] = {f: getattr(r, f).cpu() for f in ("n_iter", "status", "n_rollouts", "cost", "x")}
            del r
    same = all(torch.equal(res["rerun"][f], res[k][f]) for k in res for f in res["rerun"])
    med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
    print("median s/solve: " + ", ".join(f"{k} {v:.3f} ({med['rerun'] / v - 1:+.2%})" for k, v in med.items()) +
          f"; outcomes bitwise equal: {same}", flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
