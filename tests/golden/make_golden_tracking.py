"""Generate tests/golden/tracking.npz by running the REFERENCE's LQR / P_inf functions (test infrastructure).

Runs in the build container only (the read-only reference is mounted at /root/reference); never on the GPU
box, never imported by the product.  Writes plain data (inputs and expected outputs); no reference source is
copied into the repository.

trajectory_tracking.py imports casadi at module level (trajectory_tracking.py:2), which is not installed, so
the module itself cannot be imported.  The functions used here never touch casadi:
  compute_P_inf        trajectory_tracking.py:144-165
  solve_LQR_tracking   trajectory_tracking.py:170-203
  simulate_tracking    trajectory_tracking.py:206-216
They are compiled from the reference file's own syntax tree (ast) and executed in a namespace holding the
reference's `trajectory_generation` module contents (what the file's `from trajectory_generation import *`
provides, trajectory_tracking.py:3) -- no casadi stand-in is created.  The MPC solver (solver_mpc, :73-140)
needs IPOPT and is NOT run: its parity is pinned to the exact solution of its equality-constrained QP (see
tests/test_tracking.py).

Fixtures (main.py task_3 / task_4 inputs):
  x_opt, u_opt            trajectories_npz/acrobot_optimal_trajectory.npz (task_3 reference, main.py:101-102)
  K_reg (500,2,4)         solve_LQR_tracking(x_opt, u_opt)
  dx, x_track, u_track    simulate_tracking for x0 = x_opt[0] + dx, dx in {0.2, 0.3} (main.py:104-112)
  A_f, B_f, P_inf         compute_P_inf(A_f, B_f, Q_mpc, R_mpc) at x_f = [pi,0,0,0] (trajectory_tracking.py:31-38)

Usage:  python tests/golden/make_golden_tracking.py
"""
import ast
import contextlib
import io
import os
import shutil
import sys
import tempfile

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
FUNCS = ("compute_P_inf", "solve_LQR_tracking", "simulate_tracking")


def main():
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    scratch = tempfile.mkdtemp(prefix="gym_golden_trk_")
    shutil.copytree(os.path.join(REF, "trajectories_npz"), os.path.join(scratch, "trajectories_npz"))
    os.chdir(scratch)
    sys.path.insert(0, REF)
    import trajectory_generation as tg   # noqa: E402  (reference module)

    src = open(os.path.join(REF, "trajectory_tracking.py")).read()
    tree = ast.parse(src)
    defs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in FUNCS]
    assert sorted(d.name for d in defs) == sorted(FUNCS)
    ns = {k: getattr(tg, k) for k in dir(tg) if not k.startswith("__")}
    ns["np"] = np
    exec(compile(ast.Module(body=defs, type_ignores=[]), os.path.join(REF, "trajectory_tracking.py"), "exec"), ns)

    d = np.load(os.path.join(REF, "trajectories_npz", "acrobot_optimal_trajectory.npz"))
    x_opt, u_opt, t_ref = d["x"], d["u"], d["t"]
    K_reg = np.asarray(ns["solve_LQR_tracking"](x_opt, u_opt))
    dxs = np.array([0.2, 0.3])
    xs, us = [], []
    for dx in dxs:
        x_tr, u_tr = ns["simulate_tracking"](x_opt, u_opt, list(K_reg), x_opt[0].copy() + dx)
        xs.append(x_tr); us.append(u_tr)

    dt = tg.dt
    x_f = np.array([np.pi, 0, 0, 0]); u_f = np.array([0, 0])
    A_f, B_f = tg.discretize_linearization(*tg.Calculate_A_B_matrixes(x_f, u_f), dt)
    Q = np.diag([120.0, 100.0, 0.0001, 0.0001]); R = np.diag([1e-6, 10.0])
    with contextlib.redirect_stdout(io.StringIO()):
        P_inf = ns["compute_P_inf"](A_f, B_f, Q, R)

    np.savez_compressed(os.path.join(OUT, "tracking.npz"), x_opt=x_opt, u_opt=u_opt, t_ref=t_ref, K_reg=K_reg,
                        dx=dxs, x_track=np.array(xs), u_track=np.array(us), A_f=A_f, B_f=B_f, Q_mpc=Q, R_mpc=R,
                        P_inf=P_inf)
    print("K_reg", K_reg.shape, "x_track", np.array(xs).shape, "P_inf diag", np.diag(P_inf))


if __name__ == "__main__":
    main()
