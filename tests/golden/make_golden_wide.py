"""Golden fixtures, second set: run the REFERENCE itself on (1) wide-start lanes with gamma_0 = 1 and
(2) the parameter sets 2 / 3 of dynamics.py.

Test infrastructure only (build container; never on the GPU box; nothing in the product imports it).
Writes plain-data .npz fixtures; no reference source is copied.  Same recipe as make_golden.py
(SURVEY.md section 8(c)): MPLBACKEND=Agg, scratch CWD with trajectories_npz/, plot_armijo_line_search
stubbed (pure plotting).

wide_lanes.npz -- lanes of tests/test_gpu_parity.py::test_last_iteration_gains_and_sigma_vs_oracle (its
    160-lane x0: th ~ U(+-1.5) from default_rng(5), the first 20 lanes with w ~ U(+-2) from default_rng(6)),
    solved by the reference's newton_Algorithm with gamma_0 = 1, tol 1e-4, for max_iters = 12 and 120:
    last-iteration K and sigma, x, u, cost / sigma-norm histories, iteration count, status and the number of
    closed-loop rollouts (the reference's forward_closed_loop_update wrapped by a counter).  These pin the
    Armijo decisions (backtracking, LS failure; trajectory_generation.py:352-369) of the far-from-converged
    regime to the reference itself, not to a restatement.

pset_kats.npz -- dynamics.py:31-61 (params_2, params_3) substituted through the reference's own
    set_params (dynamics.py:117-144): the returned M, C, G, F are assembled into
    f = [qdot; M^-1 (tau_acrobot - (C + F) qdot - G)] with tau_acrobot = [0, tau2] as the module does for set 1
    (dynamics.py:150-170), lambdified, and evaluated at the 64 KAT points of kat_primitives.npz: continuous
    dynamics, one RK4 step (the formula of dynamics.py:177-195, dt = 0.02) and the Jacobians A_c, B_c.

Usage:  python tests/golden/make_golden_wide.py [--jobs 8] [--only wide|pset]
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

# lanes of the 160-lane oracle test that the reference is run on (indices into its x0)
# 0-3: initial velocities; 20-31: zero-velocity wide starts; the rest: the lanes on which two restatements (the
# C and the numpy oracle) differ most after 120 iterations, i.e. where rounding is amplified most
WIDE_LANES = (0, 1, 2, 3, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 56, 74, 80, 89, 116, 122, 143, 151)
WIDE_ITERS = (12, 120)


def wide_x0(B=160):
    """The x0 of test_last_iteration_gains_and_sigma_vs_oracle (lane 9 = NaN is not run here)."""
    x0 = np.zeros((B, 4))
    x0[:, :2] = np.random.default_rng(5).uniform(-1.5, 1.5, (B, 2))
    x0[:20, 2:] = np.random.default_rng(6).uniform(-2.0, 2.0, (20, 2))
    x0[9] = np.nan
    return x0


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


def job_wide(args):
    lane, max_iters = args
    tg = _import_reference()
    x_ref, u_ref, _ = tg.get_fully_actuated_ref()
    n_roll = [0]
    inner = tg.forward_closed_loop_update

    def counted(*a, **k):               # instrumentation only: count the Armijo trials' rollouts
        n_roll[0] += 1
        return inner(*a, **k)

    tg.forward_closed_loop_update = counted
    x0 = wide_x0()[lane]
    buf = io.StringIO()
    t0 = time.time()
    with contextlib.redirect_stdout(buf):
        x, u, K, sigma, hist = tg.newton_Algorithm(np.asarray(x0, float), x_ref, u_ref, max_iters=max_iters,
                                                   tol=1e-4, gamma_0=1.0, plot_armijo_iters=0)
    log = buf.getvalue()
    status = 1 if "Converged at iteration" in log else (2 if "Line search failed" in log else 3)
    return (lane, max_iters), dict(
        x0=x0, x=np.asarray(x), u=np.asarray(u), K=np.asarray(K), sigma=np.asarray(sigma),
        cost_hist=np.asarray(hist["cost"], float), sigma_norm_hist=np.asarray(hist["sigma_norm"], float),
        n_iter=len(hist["sigma_norm"]), status=status, n_rollouts=n_roll[0], wall_s=time.time() - t0)


def job_pset(pset):
    _import_reference()
    import sympy as sp
    import dynamics as dyn
    M, Cm, G, F = dyn.set_params(pset)
    x_vec = [dyn.theta1, dyn.theta2, dyn.theta1_dot, dyn.theta2_dot]
    u_vec = [dyn.tau1, dyn.tau2]
    qd = sp.Matrix(x_vec[2:])
    rhs = sp.Matrix([0, dyn.tau2]) - ((Cm + F) @ qd + G)
    f = sp.Matrix.vstack(qd, M.LUsolve(rhs))
    args = x_vec + u_vec
    f_fun = sp.lambdify(args, f, "numpy")
    A_fun = sp.lambdify(args, f.jacobian(x_vec), "numpy")
    B_fun = sp.lambdify(args, f.jacobian(u_vec), "numpy")
    kat = np.load(os.path.join(OUT, "kat_primitives.npz"))
    X, U = kat["X"], kat["U"]
    dt = dyn.dt

    def fc(x, u):
        return np.asarray(f_fun(*x, *u), float).reshape(4)

    out = {"f_cont": [], "f_rk4": [], "A_c": [], "B_c": []}
    for x, u in zip(X, U):
        out["f_cont"].append(fc(x, u))
        k1 = fc(x, u); k2 = fc(x + dt / 2 * k1, u); k3 = fc(x + dt / 2 * k2, u); k4 = fc(x + dt * k3, u)
        out["f_rk4"].append(x + dt * (k1 + 2 * k2 + 2 * k3 + k4) / 6.0)
        out["A_c"].append(np.asarray(A_fun(*x, *u), float))
        out["B_c"].append(np.asarray(B_fun(*x, *u), float))
    return pset, {k: np.stack(v) for k, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    if a.only in ("", "pset"):
        with ctx.Pool(2) as pool:
            res = pool.map(job_pset, (2, 3))
        kat = np.load(os.path.join(OUT, "kat_primitives.npz"))
        d = {"X": kat["X"], "U": kat["U"]}
        for pset, r in res:
            d.update({f"p{pset}_{k}": v for k, v in r.items()})
        np.savez_compressed(os.path.join(OUT, "pset_kats.npz"), **d)
        print("wrote pset_kats.npz", flush=True)
    if a.only in ("", "wide"):
        jobs = [(lane, it) for it in WIDE_ITERS for lane in WIDE_LANES]
        jobs.sort(key=lambda j: -j[1])                      # long runs first
        with ctx.Pool(a.jobs) as pool:
            res = dict(pool.map(job_wide, jobs))
        d = {"lanes": np.array(WIDE_LANES), "iters": np.array(WIDE_ITERS)}
        for it in WIDE_ITERS:
            rs = [res[(lane, it)] for lane in WIDE_LANES]
            for k in ("x0", "x", "u", "K", "sigma", "n_iter", "status", "n_rollouts", "wall_s"):
                d[f"m{it}_{k}"] = np.stack([np.asarray(r[k]) for r in rs])
            for k in ("cost_hist", "sigma_norm_hist"):
                L = max(len(r[k]) for r in rs)
                arr = np.full((len(rs), L), np.nan)
                for i, r in enumerate(rs):
                    arr[i, :len(r[k])] = r[k]
                d[f"m{it}_{k}"] = arr
            for lane, r in zip(WIDE_LANES, rs):
                print(f"max_iters={it} lane {lane}: n_iter={r['n_iter']} status={r['status']} "
                      f"rollouts={r['n_rollouts']} wall={r['wall_s']:.1f}s", flush=True)
        np.savez_compressed(os.path.join(OUT, "wide_lanes.npz"), **d)
        print("wrote wide_lanes.npz", flush=True)


if __name__ == "__main__":
    main()
