"""Golden fixture, stress set: run the REFERENCE's newton_Algorithm on selected lanes of bench.py's stress workload
(262,144 lanes, th ~ U(+-1.5) from default_rng(0), task-2 settings, max_iters 5000), to settle the lanes
on which the GPU solve and the C oracle take different Armijo decisions.

Test infrastructure only (build container; never on the GPU box; nothing in the product imports it).  Writes a
plain-data .npz fixture; no reference source is copied.  Same recipe as make_golden.py:
MPLBACKEND=Agg, scratch CWD with trajectories_npz/, plot_armijo_line_search stubbed (pure plotting).

Lanes (indices into bench.make_x0(262144, spread=1.5)), chosen from round 4's GPU solve of the whole batch
(tools/stress_parity.py -> gpurun_out/r04/stress/full.npz) against tests/golden/stress_oracle.npz:
  STATUS_FLIPS : every lane whose final status differs (GPU LS failure vs oracle convergence, or the reverse);
  MISMATCH     : the first 12 lanes (by index, <= 420 iterations) whose iteration / rollout counts differ;
  AGREE_LS     : the first 6 LS-failure lanes (<= 420 iterations) on which the two agree exactly;
  AGREE_CONV   : lanes 1, 3, 4, 5, converged, on which they agree.
Per lane the reference's own record: iteration count, status (from its log lines), closed-loop rollouts (its
forward_closed_loop_update wrapped by a counter), the cost and max|sigma| histories, and each iteration's
tightest Armijo margin min |J_new - (J + c gamma dJ)| / |J| over its trials (from its total_cost values and the
delta_J its calculate_K_and_sigma returns: instrumentation only, the algorithm is unchanged).

Usage:  python tests/golden/make_golden_stress.py [--jobs 8]
"""
import argparse
import contextlib
import io
import multiprocessing as mp
import os
import shutil
import sys
import tempfile
import time

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(OUT))

STATUS_FLIPS = (15566, 62679, 67160, 118493, 259168)
MISMATCH = (19, 35, 66, 78, 103, 149, 165, 168, 184, 270, 299, 330)
AGREE_LS = (8, 38, 39, 43, 45, 68)
AGREE_CONV = (1, 3, 4, 5)
LANES = STATUS_FLIPS + MISMATCH + AGREE_LS + AGREE_CONV


def stress_x0():
    sys.path.insert(0, ROOT)
    from bench import make_x0
    return make_x0(262144, spread=1.5)


def _import_reference():
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    scratch = tempfile.mkdtemp(prefix="gym_golden_")
    shutil.copytree(os.path.join(REF, "trajectories_npz"), os.path.join(scratch, "trajectories_npz"))
    os.chdir(scratch)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import trajectory_generation as tg  # noqa: E402
    tg.plot_armijo_line_search = lambda *a, **k: None
    return tg


def job(lane):
    x0 = stress_x0()[lane]
    tg = _import_reference()
    x_ref, u_ref, _ = tg.get_fully_actuated_ref()
    rec = {"rollouts": 0, "dJ": [], "trial_costs": []}
    fcl, tc, kas = tg.forward_closed_loop_update, tg.total_cost, tg.calculate_K_and_sigma
    in_trial = [False]

    def counted(*a, **k):               # instrumentation: count the Armijo trials' rollouts
        rec["rollouts"] += 1
        in_trial[0] = True
        return fcl(*a, **k)

    def costed(*a, **k):                # instrumentation: the cost of each trial (the call after a rollout)
        J = tc(*a, **k)
        if in_trial[0]:
            rec["trial_costs"][-1].append(float(J))
            in_trial[0] = False
        return J

    def riccati(*a, **k):               # instrumentation: each iteration's delta_J
        K, sigma, dJ = kas(*a, **k)
        rec["dJ"].append(float(dJ))
        rec["trial_costs"].append([])
        return K, sigma, dJ

    tg.forward_closed_loop_update, tg.total_cost, tg.calculate_K_and_sigma = counted, costed, riccati
    buf = io.StringIO()
    t0 = time.time()
    with contextlib.redirect_stdout(buf):
        x, u, K, sigma, hist = tg.newton_Algorithm(np.asarray(x0, float), x_ref, u_ref, max_iters=5000, tol=1e-4,
                                                   gamma_0=0.1, plot_armijo_iters=0)
    log = buf.getvalue()
    status = 1 if "Converged at iteration" in log else (2 if "Line search failed" in log else 3)
    cost = np.asarray(hist["cost"], float)          # J_0, then J after each accepted iteration
    n_iter = len(hist["sigma_norm"])
    margin = np.full(n_iter, np.inf)
    gam = 0.1
    for k in range(n_iter):
        J = cost[k]
        g = gam
        for Jn in rec["trial_costs"][k]:
            margin[k] = min(margin[k], abs(Jn - (J + 0.5 * g * rec["dJ"][k])) / max(abs(J), 1e-300))
            g *= 0.7
    return lane, dict(lane=lane, x0=x0, n_iter=n_iter, status=status, n_rollouts=rec["rollouts"], cost=cost,
                      sigma_norm=np.asarray(hist["sigma_norm"], float), margin=margin, x=np.asarray(x),
                      wall_s=time.time() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    with ctx.Pool(a.jobs) as pool:
        res = dict(pool.map(job, LANES))
    d = {"lanes": np.array(LANES), "status_flips": np.array(STATUS_FLIPS), "mismatch": np.array(MISMATCH),
         "agree_ls": np.array(AGREE_LS), "agree_conv": np.array(AGREE_CONV)}
    rs = [res[l] for l in LANES]
    for k in ("x0", "n_iter", "status", "n_rollouts", "x", "wall_s"):
        d[k] = np.stack([np.asarray(r[k]) for r in rs])
    for k in ("cost", "sigma_norm", "margin"):
        L = max(len(r[k]) for r in rs)
        arr = np.full((len(rs), L), np.nan)
        for i, r in enumerate(rs):
            arr[i, :len(r[k])] = r[k]
        d[k] = arr
    for r in rs:
        print(f"lane {r['lane']}: n_iter={r['n_iter']} status={r['status']} rollouts={r['n_rollouts']} "
              f"min margin={np.min(r['margin']):.2e} wall={r['wall_s']:.0f}s", flush=True)
    np.savez_compressed(os.path.join(OUT, "stress_ref_lanes.npz"), **d)
    print("wrote stress_ref_lanes.npz", flush=True)


if __name__ == "__main__":
    main()
