"""Golden fixture, stress tie lanes: run the REFERENCE's newton_Algorithm on the 58 stress lanes whose GPU / C-oracle
divergence carries the largest Armijo margins (>= 1e-13 at the iteration the two records part),
to pin the tie threshold of tests/stress_settle.py (TIE) to the reference itself.

Test infrastructure only (build container; never on the GPU box; nothing in the product imports it).  Writes a
plain-data .npz fixture; no reference source is copied.  Same recipe and instrumentation as make_golden_stress.py
(MPLBACKEND=Agg, scratch CWD with trajectories_npz/, plot_armijo_line_search stubbed; the
trial costs and delta_J are observed through wrappers, the algorithm is unchanged).

Lanes: indices into bench.make_x0(262144, spread=1.5), with the iteration k at which the GPU's per-iteration record
and the C oracle's part (profiles/r05/settle/settle_trials.npz, tools/stress_settle_dump.py).  The reference runs
each lane with max_iters = k + 1, i.e. iterations 0..k: enough to see which way the reference takes iteration k's
Armijo tests (a shorter max_iters changes no earlier iteration, trajectory_generation.py:329-396).  Per lane and
iteration it records the Armijo trials evaluated, the cost after the iteration (NaN on a failed line search) and the
tightest margin min |J_new - (J + c gamma dJ)| / |J| over the trials (the oracle's hist_margin definition).

Usage:  python tests/golden/make_golden_stress_ties.py [--jobs 7]
"""
import argparse
import contextlib
import io
import multiprocessing as mp
import os
import sys
import time

import numpy as np

OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, OUT)
from make_golden_stress import _import_reference, stress_x0  # noqa: E402

# (lane, k): the 58 lanes of bench.py's stress batch whose first GPU / C-oracle divergence (a different Armijo trial
# count at iteration k) has an oracle margin >= 1e-13 there (settle_trials.npz, round 5)
TIE_LANES = (
    (233548, 395), (236976, 400), (51763, 402), (146833, 402), (106919, 408), (53342, 409), (157540, 409),
    (133764, 411), (190420, 412), (132689, 413), (247790, 414), (230859, 415), (138679, 416), (180205, 419),
    (143101, 420), (5916, 424), (153526, 426), (218266, 427), (11758, 429), (220777, 434), (157903, 436),
    (60479, 437), (236814, 446), (142003, 447), (82982, 450), (147041, 452), (209562, 455), (252419, 458),
    (13171, 461), (137971, 461), (49465, 466), (166426, 468), (91950, 472), (186265, 473), (153483, 478),
    (113740, 480), (168467, 481), (105924, 490), (165665, 498), (165679, 499), (196257, 502), (144953, 503),
    (107894, 504), (168356, 508), (35085, 511), (163435, 513), (202290, 522), (167065, 525), (122116, 537),
    (18248, 544), (253842, 612), (20212, 617), (98315, 618), (97657, 620), (174589, 661), (103559, 668),
    (55002, 690), (152636, 867))


def job(arg):
    lane, k_div = arg
    x0 = stress_x0()[lane]
    tg = _import_reference()
    x_ref, u_ref, _ = tg.get_fully_actuated_ref()
    rec = {"dJ": [], "trial_costs": []}
    fcl, tc, kas = tg.forward_closed_loop_update, tg.total_cost, tg.calculate_K_and_sigma
    in_trial = [False]

    def counted(*a, **k):
        in_trial[0] = True
        return fcl(*a, **k)

    def costed(*a, **k):
        J = tc(*a, **k)
        if in_trial[0]:
            rec["trial_costs"][-1].append(float(J))
            in_trial[0] = False
        return J

    def riccati(*a, **k):
        K, sigma, dJ = kas(*a, **k)
        rec["dJ"].append(float(dJ))
        rec["trial_costs"].append([])
        return K, sigma, dJ

    tg.forward_closed_loop_update, tg.total_cost, tg.calculate_K_and_sigma = counted, costed, riccati
    buf = io.StringIO()
    t0 = time.time()
    with contextlib.redirect_stdout(buf):
        _, _, _, _, hist = tg.newton_Algorithm(np.asarray(x0, float), x_ref, u_ref, max_iters=k_div + 1, tol=1e-4,
                                               gamma_0=0.1, plot_armijo_iters=0)
    log = buf.getvalue()
    status = 1 if "Converged at iteration" in log else (2 if "Line search failed" in log else 3)
    J = np.asarray(hist["cost"], float)               # J_0, then J after each accepted iteration
    n = len(rec["dJ"])
    trials = np.array([len(t) for t in rec["trial_costs"]], np.int64)
    margin = np.full(n, np.inf)
    cost_after = np.full(n, np.nan)
    for i in range(n):
        g = 0.1
        for Jn in rec["trial_costs"][i]:
            margin[i] = min(margin[i], abs(Jn - (J[i] + 0.5 * g * rec["dJ"][i])) / max(abs(J[i]), 1e-300))
            g *= 0.7
        if i + 1 < len(J):
            cost_after[i] = J[i + 1]
    return lane, dict(lane=lane, k=k_div, n_iter=n, status=status, trials=trials, cost_after=cost_after,
                      margin=margin, wall_s=time.time() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=7)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    t0 = time.time()
    res = {}
    # longest first, so the pool ends together
    work = sorted(TIE_LANES, key=lambda lk: -lk[1])
    with ctx.Pool(a.jobs) as pool:
        for lane, r in pool.imap_unordered(job, work):
            res[lane] = r
            print(f"lane {lane}: k={r['k']} ran {r['n_iter']} status={r['status']} trials[k]={r['trials'][-1]} "
                  f"margin[k]={r['margin'][-1]:.3e} wall={r['wall_s']:.0f}s ({len(res)}/{len(work)}, "
                  f"{time.time() - t0:.0f}s)", flush=True)
    lanes = [lk[0] for lk in TIE_LANES]
    rs = [res[l] for l in lanes]
    L = max(r["n_iter"] for r in rs)
    d = {"lanes": np.array(lanes), "k": np.array([r["k"] for r in rs]),
         "n_iter": np.array([r["n_iter"] for r in rs]), "status": np.array([r["status"] for r in rs]),
         "wall_s": np.array([r["wall_s"] for r in rs])}
    for key, fill, dt in (("trials", -1, np.int64), ("cost_after", np.nan, float), ("margin", np.nan, float)):
        arr = np.full((len(rs), L), fill, dtype=dt)
        for i, r in enumerate(rs):
            arr[i, :len(r[key])] = r[key]
        d[key] = arr
    np.savez_compressed(os.path.join(OUT, "stress_tie_lanes.npz"), **d)
    print(f"wrote stress_tie_lanes.npz ({time.time() - t0:.0f} s)", flush=True)


if __name__ == "__main__":
    main()
