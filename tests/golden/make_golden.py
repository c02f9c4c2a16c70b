"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Test infrastructure only. This script runs in the build container (where the read-only
reference is mounted at /root/reference); it never runs on the GPU box, and nothing in the
product imports it. It writes plain-data .npz fixtures (inputs and expected outputs); no
reference source is copied.

Recipe:
  * MPLBACKEND=Agg, sys.path.insert(0, REF), chdir into a scratch dir holding a copy of
    trajectories_npz/ (get_fully_actuated_ref loads a CWD-relative path,
    trajectory_generation.py:513);
  * trajectory_generation.plot_armijo_line_search is replaced by a no-op (pure plotting,
    trajectory_generation.py:254-296; it also runs 200 extra rollouts per plotted iteration);
  * newton_Algorithm is called with main.task_2's arguments (main.py:65-71).

Usage:  python tests/golden/make_golden.py [--jobs 8]
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


def _solve(tg, x0, x_ref, u_ref, max_iters, tol, gamma_0, keep_x_iters=(0, 1, 2)):
    buf = io.StringIO()
    t0 = time.time()
    with contextlib.redirect_stdout(buf):
        x, u, K, sigma, hist = tg.newton_Algorithm(
            np.asarray(x0, dtype=float), x_ref, u_ref, max_iters=max_iters, tol=tol,
            gamma_0=gamma_0, plot_armijo_iters=0)
    wall = time.time() - t0
    log = buf.getvalue()
    failed = "Line search failed" in log
    converged = "Converged at iteration" in log
    n_iter = len(hist["sigma_norm"])  # outer iterations executed (incl. a final failed one)
    xs = hist["x_trajs"]
    keep = sorted(set(i for i in keep_x_iters if i < len(xs)) | {len(xs) - 1})
    return dict(
        x=np.asarray(x), u=np.asarray(u), K=np.asarray(K), sigma=np.asarray(sigma),
        cost_hist=np.asarray(hist["cost"], dtype=float),
        sigma_norm_hist=np.asarray(hist["sigma_norm"], dtype=float),
        x_hist_idx=np.asarray(keep), x_hist=np.stack([xs[i] for i in keep]),
        sigma_first=np.asarray(hist["sigmas"][0]),
        n_iter=np.int64(n_iter), status=np.int64(1 if converged else (2 if failed else 3)),
        wall_s=np.float64(wall),
    )


# --------------------------------------------------------------------------------------
# jobs
# --------------------------------------------------------------------------------------

def job_task2(_):
    tg = _import_reference()
    x_ref, u_ref, t_ref = tg.get_fully_actuated_ref()
    r = _solve(tg, np.zeros(4), x_ref, u_ref, 5000, 1e-4, 0.1)
    r.update(x_ref=x_ref, u_ref=u_ref, t_ref=t_ref, x0=np.zeros(4))
    return "task2_solve", r


def job_lane(args):
    name, x0, max_iters = args
    tg = _import_reference()
    x_ref, u_ref, _ = tg.get_fully_actuated_ref()
    r = _solve(tg, x0, x_ref, u_ref, max_iters, 1e-4, 0.1)
    r["x0"] = np.asarray(x0, dtype=float)
    return name, r


def job_task1(_):
    tg = _import_reference()
    x_e1, u_e1 = tg.compute_equilibrium(np.array([0.0, 0.0]), (0.1, -0.1))
    x_e2, u_e2 = tg.compute_equilibrium(np.array([0.5, 0.5]), (0.35, -0.35))
    t_ref, x_ref, u_ref = tg.define_reference_piecewise(10.0, x_e1, x_e2, u_e1, u_e2)
    r = _solve(tg, x_e1.copy(), x_ref, u_ref, 5000, 1e-4, 0.05)
    r.update(x_ref=x_ref, u_ref_full=u_ref, t_ref=t_ref, x0=x_e1.copy(),
             x_e1=x_e1, x_e2=x_e2, u_e1=u_e1, u_e2=u_e2)
    return "task1_solve", r


def job_kats(_):
    """Known-answer vectors for the per-stage primitives (dynamics.py, trajectory_generation.py)."""
    tg = _import_reference()
    import dynamics as dyn
    rng = np.random.default_rng(1234)
    n = 64
    X = np.empty((n, 4)); U = np.empty((n, 2))
    X[:, :2] = rng.uniform(-np.pi, np.pi, (n, 2)); X[:, 2:] = rng.uniform(-8, 8, (n, 2))
    U[:] = rng.uniform(-20, 20, (n, 2))
    X[0] = [.1, .2, .3, .4]; U[0] = [0., 1.5]            # SURVEY 8(a) KAT point
    X[1] = [0, 0, 0, 0]; U[1] = [0, 0]
    X[2] = [np.pi, 0, 0, 0]; U[2] = [0, 0]                 # upright (trajectory_tracking.py:33)
    X[3, :2] = [40.0, -37.5]                               # large angles
    X[4, :2] = [1e3, -2e3]                                 # very large angles (range reduction)
    X[5, 2:] = [25.0, -30.0]                               # fast spin
    fc = np.stack([dyn.continuous_dynamics(X[i], U[i]) for i in range(n)])
    fd = np.stack([dyn.dynamics(X[i], U[i]) for i in range(n)])
    A = np.empty((n, 4, 4)); B = np.empty((n, 4, 2))
    for i in range(n):
        A[i], B[i] = dyn.Calculate_A_B_matrixes(X[i], U[i])
    Ad = np.empty((n, 4, 4)); Bd = np.empty((n, 4, 2))
    for i in range(n):
        Ad[i], Bd[i] = tg.discretize_linearization(A[i], B[i], dyn.dt)

    # stage-cost derivatives with general (non-diagonal) weights
    xr = rng.normal(size=(n, 4)); ur = rng.normal(size=(n, 2))
    Mq = rng.normal(size=(4, 4)); Qg = Mq @ Mq.T + np.eye(4)
    Mr = rng.normal(size=(2, 2)); Rg = Mr @ Mr.T + np.eye(2)
    Mt = rng.normal(size=(4, 4)); QTg = Mt @ Mt.T + np.eye(4)
    l = np.empty(n); gx = np.empty((n, 4)); gu = np.empty((n, 2)); lT = np.empty(n); gT = np.empty((n, 4))
    for i in range(n):
        l[i], gx[i], gu[i], _, _ = tg.derivatives_Cost(X[i], xr[i], U[i], ur[i], Qg, Rg)
        lT[i], gT[i], _ = tg.derivatives_Cost(X[i], xr[i], U[i], ur[i], None, None, Q_T=QTg, terminal=True)
    return "kat_primitives", dict(X=X, U=U, f_cont=fc, f_rk4=fd, A_c=A, B_c=B, A_d=Ad, B_d=Bd, dt=np.float64(dyn.dt),
                                  xr=xr, ur=ur, Qg=Qg, Rg=Rg, QTg=QTg, l=l, gx=gx, gu=gu, lT=lT, gT=gT)


def job_iteration(_):
    """Intermediates of single Newton iterations."""
    tg = _import_reference()
    x_ref, u_ref, _ = tg.get_fully_actuated_ref()
    out = {}
    # iteration-0 point of task 2: open-loop rollout with u = 0 (trajectory_generation.py:311-312)
    u0 = np.zeros_like(u_ref)
    x0 = tg.simulate_open_loop(np.zeros(4), u0)
    # a mid-solve point: 40 Newton iterations from a non-zero start
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        xm, um, _, _, _ = tg.newton_Algorithm(np.array([0.3, -0.2, 0.0, 0.0]), x_ref, u_ref, max_iters=40,
                                              tol=1e-12, gamma_0=0.1, plot_armijo_iters=0)
    for tag, (xt, ut) in {"it0": (x0, u0), "mid": (xm, um)}.items():
        lam = tg.compute_costate_trajectory(xt, ut, x_ref, u_ref)
        lists = tg.build_stage_lists(xt, ut, x_ref, u_ref, lam)
        K, sig, dJ = tg.calculate_K_and_sigma(*lists)
        xn, un = tg.forward_closed_loop_update(xt, ut, K, sig, gamma=0.1)
        xn1, un1 = tg.forward_closed_loop_update(xt, ut, K, sig, gamma=1.0)
        out.update({
            f"{tag}_x": xt, f"{tag}_u": ut, f"{tag}_lambda": np.asarray(lam),
            f"{tag}_A_d": np.asarray(lists[0]), f"{tag}_B_d": np.asarray(lists[1]),
            f"{tag}_q": np.asarray(lists[5]), f"{tag}_r": np.asarray(lists[6]),
            f"{tag}_QT": lists[7], f"{tag}_qT": lists[8],
            f"{tag}_K": np.asarray(K), f"{tag}_sigma": np.asarray(sig), f"{tag}_dJ": np.float64(dJ),
            f"{tag}_cost": np.float64(tg.total_cost(xt, ut, x_ref, u_ref, tg.Q, tg.R, tg.Q_T)),
            f"{tag}_xn01": xn, f"{tag}_un01": un,
            f"{tag}_cost01": np.float64(tg.total_cost(xn, un, x_ref, u_ref, tg.Q, tg.R, tg.Q_T)),
            f"{tag}_xn1": xn1, f"{tag}_un1": un1,
            f"{tag}_cost1": np.float64(tg.total_cost(xn1, un1, x_ref, u_ref, tg.Q, tg.R, tg.Q_T)),
        })
    out.update(x_ref=x_ref, u_ref=u_ref)
    # general (unstructured) Riccati lists: dense A, B, S, non-diagonal Q, R (calculate_K_and_sigma:183-216)
    rng = np.random.default_rng(77)
    T = 24
    A = [np.eye(4) + 0.1 * rng.normal(size=(4, 4)) for _ in range(T)]
    B = [0.1 * rng.normal(size=(4, 2)) for _ in range(T)]
    Ql, Rl, Sl, ql, rl = [], [], [], [], []
    for _ in range(T):
        M = rng.normal(size=(4, 4)); Ql.append(M @ M.T + np.eye(4))
        M = rng.normal(size=(2, 2)); Rl.append(M @ M.T + np.eye(2))
        Sl.append(0.1 * rng.normal(size=(2, 4)))
        ql.append(rng.normal(size=4)); rl.append(rng.normal(size=2))
    M = rng.normal(size=(4, 4)); QT = M @ M.T + np.eye(4); qT = rng.normal(size=4)
    K, sig, dJ = tg.calculate_K_and_sigma(A, B, Ql, Rl, Sl, ql, rl, QT, qT)
    out.update(gen_A=np.asarray(A), gen_B=np.asarray(B), gen_Q=np.asarray(Ql), gen_R=np.asarray(Rl),
               gen_S=np.asarray(Sl), gen_q=np.asarray(ql), gen_r=np.asarray(rl), gen_QT=QT, gen_qT=qT,
               gen_K=np.asarray(K), gen_sigma=np.asarray(sig), gen_dJ=np.float64(dJ))
    # simulate_open_loop with a random control sequence
    uu = rng.uniform(-3, 3, size=(500, 2))
    out.update(sim_x0=np.array([0.2, -0.4, 0.5, -1.0]), sim_u=uu,
               sim_x=tg.simulate_open_loop(np.array([0.2, -0.4, 0.5, -1.0]), uu))
    return "newton_iteration", out


def _lane_jobs():
    jobs = []
    # headline distribution: x0 = [th1, th2, 0, 0], th ~ U(-0.5, 0.5)
    for s in range(6):
        th = np.random.default_rng(s).uniform(-0.5, 0.5, 2)
        jobs.append((f"lane_u05_s{s}", np.array([th[0], th[1], 0.0, 0.0]), 5000))
    # stress variants: wider angles, initial velocities -> backtracking / LS failure
    for s in (10, 11):
        th = np.random.default_rng(s).uniform(-1.5, 1.5, 2)
        jobs.append((f"lane_u15_s{s}", np.array([th[0], th[1], 0.0, 0.0]), 5000))
    for s in (12, 13):
        th = np.random.default_rng(s).uniform(-np.pi, np.pi, 2)
        jobs.append((f"lane_upi_s{s}", np.array([th[0], th[1], 0.0, 0.0]), 900))
    for s in (14, 15):
        r = np.random.default_rng(s)
        th = r.uniform(-0.5, 0.5, 2); w = r.uniform(-2, 2, 2)
        jobs.append((f"lane_vel_s{s}", np.array([th[0], th[1], w[0], w[1]]), 900))
    return jobs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    tasks = [(job_kats, None), (job_iteration, None), (job_task2, None), (job_task1, None)]
    tasks += [(job_lane, j) for j in _lane_jobs()]
    if a.only:
        tasks = [t for t in tasks if a.only in t[0].__name__ or (t[1] and a.only in t[1][0])]
    with mp.get_context("spawn").Pool(a.jobs) as pool:
        res = [pool.apply_async(f, (arg,)) for f, arg in tasks]
        results = [r.get() for r in res]
    lanes = {}
    for name, d in results:
        if name.startswith("lane_"):
            lanes[name] = d
            print(f"{name}: n_iter={int(d['n_iter'])} status={int(d['status'])} "
                  f"J={d['cost_hist'][-1]:.6f} wall={float(d['wall_s']):.1f}s", flush=True)
            continue
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **d)
        extra = f" n_iter={int(d['n_iter'])} status={int(d['status'])}" if "n_iter" in d else ""
        print(f"wrote {name}.npz{extra}", flush=True)
    if lanes:
        names = sorted(lanes)
        packed = {"names": np.array(names)}
        for k in ("x0", "x", "u", "K", "sigma", "cost_hist", "sigma_norm_hist", "n_iter", "status", "wall_s"):
            vals = [lanes[n][k] for n in names]
            if k in ("cost_hist", "sigma_norm_hist"):
                L = max(len(v) for v in vals)
                arr = np.full((len(vals), L), np.nan)
                for i, v in enumerate(vals):
                    arr[i, :len(v)] = v
                packed[k] = arr
            else:
                packed[k] = np.stack(vals)
        np.savez_compressed(os.path.join(OUT, "lanes.npz"), **packed)
        print("wrote lanes.npz", flush=True)


if __name__ == "__main__":
    main()
