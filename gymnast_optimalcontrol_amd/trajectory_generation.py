"""Drop-in for the reference's ``trajectory_generation.py`` hot path, computed by the HIP engine.

Same module constants (T, N, nu, nx, Q, R, Q_T; :8-18), same functions with the reference's
argument order, defaults, return structure and error behaviour:

  simulate_open_loop (:74)          -> gym_rollout_open_loop
  derivatives_Cost (:89)            -> gym_stage_cost_derivs
  stage_blocks_and_affine (:116), terminal_blocks (:131)   (via derivatives_Cost)
  compute_costate_trajectory (:138) -> gym_backward_sweep (costate output)
  discretize_linearization (:161)   (4x4 host glue; the same map is fused in the kernels)
  build_stage_lists (:166)          -> gym_linearize
  calculate_K_and_sigma (:183)      -> gym_riccati_general
  forward_closed_loop_update (:218) -> gym_closed_loop
  total_cost (:231)                 -> gym_total_cost
  plot_armijo_line_search (:254)    -> gym_gamma_sweep (the 200-rollout curve) + the line-search figure
  generate_report_graphs (:405)     report figures from the results and history (matplotlib, optional);
                                    plot_results (called by main.task_1, absent from the reference) = the same
  newton_Algorithm (:298)           -> gym_newton_init / gym_newton_iteration / gym_newton_finalize
  get_fully_actuated_ref (:511), compute_equilibrium (:22), define_reference_piecewise (:41)
                                    (problem setup on the host, as in the reference)

Like the reference, the weights are read from this module's globals Q, R, Q_T at call time.
Batched variants (``*_batch``) take stacks of lanes and return device tensors.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .dynamics import (Calculate_A_B_matrixes, continuous_dynamics, dt, dynamics, engine, ni, ns,  # noqa: F401
                       set_params, set_params_numeric, use_params)
from .engine import Weights
from .params import MAX_LINE_SEARCH_ITERS
from .solver import BatchedNewtonSolver, SolveResult, newton_solve_batch  # noqa: F401

T = 10.0
N = int(T / dt) + 1
nu = 2
nx = 4

Q = np.diag([130.0, 30.0, 0.0001, 0.0001])
R = np.diag([1e-6, 1.5])
Q_T = np.diag([130, 130., 1., 1.0])


def _eng():
    e = engine()
    e.set_weights(Weights.from_matrices(Q, R, Q_T))
    return e


# ------------------------------------------------------------------------------ problem setup
def compute_equilibrium(u_target, theta_guess):
    """Solve G(theta1, theta2) = u_target (:22-39) with scipy's hybrid root finder."""
    from scipy.optimize import root
    _, _, G, _ = set_params_numeric(1)          # the numbers of set_params(1)'s G, without sympy
    u_target = np.asarray(u_target, dtype=float)
    sol = root(lambda th: np.asarray(G(th[0], th[1]), dtype=float).reshape(-1) - u_target, theta_guess,
               method="hybr")
    if not sol.success:
        raise RuntimeError("Root finder failed: " + sol.message)
    return np.array([sol.x[0], sol.x[1], 0.0, 0.0]), np.array(u_target, dtype=float).reshape(-1)


def define_reference_piecewise(T, x_e1, x_e2, u_e1, u_e2):
    """Two constant segments: x_e1 for t < T/2, x_e2 after (:41-58)."""
    Nn = int(T / dt) + 1
    t_ref = np.linspace(0.0, T, Nn)
    first = (t_ref < T / 2.0)[:, None]
    x_ref = np.where(first, np.asarray(x_e1, float)[None], np.asarray(x_e2, float)[None])
    u_ref = np.where(first, np.asarray(u_e1, float)[None], np.asarray(u_e2, float)[None])
    return t_ref, x_ref, u_ref


def get_fully_actuated_ref(path="trajectories_npz/fully_actuated_trajectory.npz"):
    """Task-2 reference (:511-518): x_ref, 2*[0, u_fa[:,1]], time.  ``path`` is CWD-relative as in the reference."""
    data = np.load(path)
    u_ref = np.zeros(data["u"].shape)
    u_ref[:, 1] = data["u"][:, 1]
    return data["x"], np.multiply(u_ref, 2), data["time"]


# ---------------------------------------------------------------------------- stage primitives
def derivatives_Cost(x, x_ref, u, u_ref, Q, R, Q_T=None, terminal=False):
    """Stage (l, q, r, 2Q, 2R) or terminal (l_T, q_T, 2Q_T) cost derivatives (:89-114)."""
    e = engine()
    if not terminal:
        l, gx, gu = e.stage_cost_derivs(np.asarray(x, float), np.asarray(x_ref, float), np.asarray(u, float),
                                        np.asarray(u_ref, float), Q, R, terminal=False)
        return float(l[0]), gx[0].cpu().numpy(), gu[0].cpu().numpy(), 2 * Q, 2 * R
    l, gx, _ = e.stage_cost_derivs(np.asarray(x, float), np.asarray(x_ref, float), None, None, Q_T, None,
                                   terminal=True)
    return float(l[0]), gx[0].cpu().numpy(), 2 * Q_T


def stage_blocks_and_affine(x, u, x_ref, u_ref, Q, R, A, B, lambda_next):
    """Gauss-Newton stage blocks (Q_t, R_t, S_t = 0, q_t, r_t) (:116-129)."""
    _, grad_x, grad_u, hess_xx, hess_uu = derivatives_Cost(x, x_ref, u, u_ref, Q, R, terminal=False)
    return hess_xx, hess_uu, np.zeros((u.shape[0], x.shape[0])), grad_x, grad_u


def terminal_blocks(x_T, x_ref_T, Q_T):
    """(Q_T block, q_T) (:131-136)."""
    _, grad_xT, hess_xx = derivatives_Cost(x_T, x_ref_T, np.zeros(nu), np.zeros(nu), Q=None, R=None, Q_T=Q_T,
                                           terminal=True)
    return hess_xx, grad_xT


def discretize_linearization(Ac, Bc, dt):
    """Forward-Euler A_d = I + dt A_c, B_d = dt B_c (:161-164)."""
    return np.eye(Ac.shape[0]) + dt * Ac, dt * Bc


# ------------------------------------------------------------------------- trajectory functions
def _zeros_refs(Nn):
    return np.zeros((Nn, 4)), np.zeros((Nn - 1, 2))


def simulate_open_loop(x0, u_traj):
    """Roll x0 forward under u_traj with RK4 (:74-87) -> (len(u)+1, nx)."""
    u_traj = np.asarray(u_traj, dtype=float)
    xr, ur = _zeros_refs(u_traj.shape[0] + 1)
    x, _ = _eng().rollout_open_loop(np.asarray(x0, float).reshape(1, 4), u_traj[None], xr, ur)
    return x[0].cpu().numpy()


def compute_costate_trajectory(x_traj, u_traj, x_ref, u_ref):
    """Costates lambda_N = 2 Q_T dx_N, lambda_t = 2 Q dx_t + A_d^T lambda_{t+1} (:138-159) -> list of N (4,)."""
    Nn = x_traj.shape[0]
    _, _, _, _, lam = _eng().backward(np.asarray(x_traj, float)[None], np.asarray(u_traj, float)[None][:, :Nn - 1],
                                      np.asarray(x_ref, float)[:Nn], np.asarray(u_ref, float)[:Nn - 1],
                                      want_lambda=True, check_gains=False)
    lam = lam[0].cpu().numpy()
    return [lam[t] for t in range(Nn)]


def build_stage_lists(x_traj, u_traj, x_ref, u_ref, lambda_seq):
    """Per-stage A_d, B_d, Q_t, R_t, S_t, q_t, r_t and the terminal blocks (:166-181)."""
    Nn = x_traj.shape[0]
    Ad, Bd, q, r, qT = _eng().linearize(np.asarray(x_traj, float)[None], np.asarray(u_traj, float)[None][:, :Nn - 1],
                                        np.asarray(x_ref, float)[:Nn], np.asarray(u_ref, float)[:Nn - 1])
    Ad, Bd, q, r, qT = (a[0].cpu().numpy() for a in (Ad, Bd, q, r, qT))
    Tn = Nn - 1
    return ([Ad[t] for t in range(Tn)], [Bd[t] for t in range(Tn)], [2 * Q for _ in range(Tn)],
            [2 * R for _ in range(Tn)], [np.zeros((nu, nx)) for _ in range(Tn)], [q[t] for t in range(Tn)],
            [r[t] for t in range(Tn)], 2 * Q_T, qT)


def calculate_K_and_sigma(A_list, B_list, Q_list, R_list, S_list, q_list, r_list, Q_T_block, q_T):
    """Backward Riccati recursion on general stage data (:183-216) -> (K list, sigma list, dJ)."""
    K, sig, dJ = engine().riccati_general(np.asarray(A_list)[None], np.asarray(B_list)[None], np.asarray(Q_list)[None],
                                          np.asarray(R_list)[None], np.asarray(S_list)[None], np.asarray(q_list)[None],
                                          np.asarray(r_list)[None], np.asarray(Q_T_block)[None],
                                          np.asarray(q_T)[None])
    K, sig = K[0].cpu().numpy(), sig[0].cpu().numpy()
    return [K[t] for t in range(K.shape[0])], [sig[t] for t in range(sig.shape[0])], float(dJ[0])


def forward_closed_loop_update(x_traj, u_traj, K, sigma, gamma=1.0):
    """u_new = u + K (x_new - x) + gamma sigma, RK4 rollout (:218-229) -> (x_new, u_new)."""
    Nn = x_traj.shape[0]
    xr, ur = _zeros_refs(Nn)
    xn, un, _ = _eng().closed_loop(np.asarray(x_traj, float)[None], np.asarray(u_traj, float)[None][:, :Nn - 1],
                                   np.asarray(K, float)[None], np.asarray(sigma, float)[None], float(gamma), xr, ur)
    u_new = np.asarray(u_traj, dtype=float).copy()
    u_new[:Nn - 1] = un[0].cpu().numpy()
    return xn[0].cpu().numpy(), u_new


def total_cost(x_traj, u_traj, x_ref, u_ref, Q, R, Q_T):
    """J = sum_t dx'Q dx + du'R du + dx_N' Q_T dx_N (:231-252)."""
    Nn = x_traj.shape[0]
    J = engine().total_cost(np.asarray(x_traj, float)[None], np.asarray(u_traj, float)[None][:, :Nn - 1],
                            np.asarray(x_ref, float)[:Nn], np.asarray(u_ref, float)[:Nn - 1], Q, R, Q_T)
    return float(J[0])


def armijo_steps(gamma_0, beta, n):
    """The Armijo trial step sizes gamma_0, gamma_0 beta, ... as the reference forms them: gamma_i *= beta,
    sequentially (:365) -- bit-identical to the solver kernels' (beta ** i would round differently)."""
    g = [float(gamma_0)]
    for _ in range(n - 1):
        g.append(g[-1] * beta)
    return np.array(g)


def plot_armijo_line_search(iteration, x_traj, u_traj, K, sigma, cost_current, x_ref, u_ref, delta_J,
                            gamma_accepted, stepsizes_tested, costs_tested, c=0.5, beta=0.7):
    """Armijo line-search report of one iteration (:254-296).

    The 200-point curve J(gamma) along the descent direction (:256-264; 200 closed-loop rollouts in the
    reference) is one gym_gamma_sweep launch; the figure is the reference's (actual cost, first-order model
    J + gamma dJ, Armijo line J + c gamma dJ, the tested and the accepted step sizes), drawn when matplotlib
    is importable.  Returns the curve data {steps, costs, linear_approx, armijo_line} as well."""
    max_step = max(1.25, max(stepsizes_tested) * 1.3 if stepsizes_tested else 1.25)
    steps = np.linspace(0, max_step, 200)
    x_traj = np.asarray(x_traj, dtype=float)
    Nn = x_traj.shape[0]
    costs = _eng().gamma_sweep(x_traj[None], np.asarray(u_traj, dtype=float)[None][:, :Nn - 1],
                               np.asarray(K, dtype=float)[None], np.asarray(sigma, dtype=float)[None], steps,
                               np.asarray(x_ref, dtype=float)[:Nn], np.asarray(u_ref, dtype=float)[:Nn - 1])
    costs = costs[0].cpu().numpy()
    curve = {"steps": steps, "costs": costs, "linear_approx": cost_current + delta_J * steps,
             "armijo_line": cost_current + c * delta_J * steps}
    _draw_armijo(iteration, curve, cost_current, delta_J, gamma_accepted, stepsizes_tested, costs_tested, c, beta,
                 max_step)
    return curve


_NON_INTERACTIVE = ("agg", "pdf", "ps", "svg", "cairo", "template")


def _pyplot():
    """matplotlib.pyplot, or None: the report figures are optional, the computed data is the result."""
    try:
        import matplotlib.pyplot as plt
    except ImportError:
        return None
    return plt


def _show(plt):
    import matplotlib
    if matplotlib.get_backend().lower() not in _NON_INTERACTIVE:
        plt.show()


def _draw_armijo(iteration, curve, cost_current, delta_J, gamma_accepted, stepsizes_tested, costs_tested, c, beta,
                 max_step):
    """The line-search figure of :266-296: the cost along the direction, its first-order model, the Armijo line,
    the tested step sizes and the accepted one."""
    plt = _pyplot()
    if plt is None:
        return
    fig, ax = plt.subplots(num=f"Armijo line search, iteration {iteration}", figsize=(12, 7), clear=True)
    for key, style, label in (("costs", "-", r"$J(\gamma)$ along the Newton direction"),
                              ("linear_approx", "--", r"$J_k + \gamma\,\Delta J$"),
                              ("armijo_line", ":", rf"$J_k + c\,\gamma\,\Delta J$ (c = {c})")):
        ax.plot(curve["steps"], curve[key], style, linewidth=2.2, label=label)
    if stepsizes_tested and costs_tested:
        ax.scatter(stepsizes_tested, costs_tested, marker="*", s=140, zorder=5, label=rf"trials ($\beta$ = {beta})")
        ax.scatter([gamma_accepted], [costs_tested[-1]], s=190, facecolors="none", edgecolors="k", linewidths=2,
                   zorder=6, label=rf"accepted $\gamma$ = {gamma_accepted:.4f}")
    ax.set(xlabel=r"step size $\gamma$", ylabel="cost J", xlim=(0, max_step),
           title=f"iteration {iteration}: J = {cost_current:.4f}, expected reduction {delta_J:.2e}")
    ax.grid(alpha=0.3)
    ax.legend(loc="best")
    fig.tight_layout()
    _show(plt)


def report_iterations(n_trajs: int) -> list:
    """Iterations whose trajectories the report overlays (:440-448): 0, 1, 5, 10, 100 where they exist plus five
    evenly spaced ones, ascending."""
    fixed = [i for i in (0, 1, 5, 10, 100) if i < n_trajs]
    even = np.linspace(0, n_trajs - 1, 5, dtype=int).tolist() if n_trajs else []
    return sorted(set(fixed) | set(even))


def generate_report_graphs(t_ref, x_ref, u_ref, x_opt, u_opt, history):
    """The report figures of :405-509 from a solve's results and ``history`` (newton_Algorithm's, or a batched
    lane's: SolveResult.x_trajs / hist_cost / hist_smax assembled into the same keys).

    Four figures: optimal angles / torques against the desired curves; intermediate trajectories (the
    iterations of ``report_iterations``); sigma_t of tau2 at the first and the last iterations; cost and
    max|sigma| per iteration on log axes.  Drawn when matplotlib is importable (shown on interactive backends);
    returns the plotted data either way."""
    t_ref = np.asarray(t_ref, float)
    x_ref, x_opt, u_opt = (np.asarray(a, float) for a in (x_ref, x_opt, u_opt))
    u_ref = np.asarray(u_ref, float)
    u_ref = u_ref[:-1] if u_ref.shape[0] == t_ref.shape[0] else u_ref
    shown = report_iterations(len(history["x_trajs"]))
    # the reference's selection (:476-477); a batched lane's history holds sigma only at the iterations it
    # recorded (None elsewhere)
    sig_its = sorted({i for i in (0, 1, 2, len(history["sigmas"]) - 1)
                      if 0 <= i < len(history["sigmas"]) and history["sigmas"][i] is not None})
    data = {"iterations_shown": shown, "sigma_iterations": sig_its,
            "sigma_tau2": {i: np.asarray(history["sigmas"][i], float).reshape(-1, 2)[:, 1] for i in sig_its},
            "cost": np.asarray(history["cost"], float), "sigma_norm": np.asarray(history["sigma_norm"], float)}
    plt = _pyplot()
    if plt is None:
        return data
    tu = t_ref[:-1]
    fig, (a0, a1) = plt.subplots(2, 1, num="optimal trajectory vs desired", figsize=(10, 8), clear=True)
    for j, col in ((0, "tab:blue"), (1, "tab:red")):
        a0.plot(t_ref, x_opt[:, j], color=col, linewidth=2, label=rf"$\theta_{j + 1}$ optimal")
        a0.plot(t_ref, x_ref[:, j], color=col, linestyle="--", alpha=0.5, label=rf"$\theta_{j + 1}$ desired")
        a1.step(tu, u_opt[:, j], color=("tab:green", "tab:purple")[j], label=rf"$\tau_{j + 1}$ optimal")
        a1.step(tu, u_ref[:, j], color=("tab:green", "tab:purple")[j], linestyle="--", alpha=0.5,
                label=rf"$\tau_{j + 1}$ desired")
    a1.axhline(0.0, color="k", linewidth=1, alpha=0.5)
    a0.set(ylabel="angle [rad]", title="optimal trajectory vs desired curve")
    a1.set(ylabel="torque [Nm]", xlabel="time [s]")
    fig2, axes = plt.subplots(2, 1, num="intermediate trajectories", figsize=(10, 7), clear=True)
    for j, ax in enumerate(axes):
        for i in shown:
            ax.plot(t_ref, np.asarray(history["x_trajs"][i])[:, j], alpha=0.4, label=f"iter {i}")
        ax.plot(t_ref, x_ref[:, j], "k--", linewidth=2, label="desired")
        ax.set(ylabel=rf"$\theta_{j + 1}$ [rad]")
    axes[0].set_title("intermediate trajectories vs desired")
    axes[1].set_xlabel("time [s]")
    fig3, a3 = plt.subplots(num="descent direction", figsize=(10, 5), clear=True)
    for i, sg in data["sigma_tau2"].items():
        a3.plot(tu, sg, label=rf"iter {i}: $\sigma_t$ ($\tau_2$)")
    a3.set(xlabel="time [s]", ylabel="correction", title=r"descent direction $\sigma_t$ of $\tau_2$")
    fig4, (b0, b1) = plt.subplots(1, 2, num="convergence", figsize=(12, 5), clear=True)
    b0.semilogy(np.arange(len(data["cost"])), data["cost"], "o-", markersize=3)
    b0.set(xlabel="iteration", ylabel="J", title="cost along iterations")
    b1.semilogy(np.arange(1, len(data["sigma_norm"]) + 1), data["sigma_norm"], "o-", markersize=3, color="tab:red")
    b1.set(xlabel="iteration", ylabel=r"$\|\sigma\|_\infty$", title="norm of the descent direction")
    for f, axs in ((fig, (a0, a1)), (fig2, axes), (fig3, (a3,)), (fig4, (b0, b1))):
        for ax in axs:
            ax.grid(True, alpha=0.3)
            if ax.get_legend_handles_labels()[0] and ax not in (b0, b1):
                ax.legend(fontsize=9)
        f.tight_layout()
    data["figures"] = [fig, fig2, fig3, fig4]
    _show(plt)
    return data


# main.task_1 calls tg.plot_results (main.py:49), which the reference module does not define (task 1 stops there
# with AttributeError); here it draws the same report.
plot_results = generate_report_graphs


# ------------------------------------------------------------------------------ the solver
def newton_Algorithm(x0, x_ref, u_ref, max_iters, tol=1e-6, beta=0.7, c=0.5, gamma_0=1, plot_armijo_iters=10,
                     verbose=True):
    """Regularised Newton's method for optimal control with Armijo line search (:298-398).

    Returns (x_traj (N,4), u_traj (N-1,2), K (list of (2,4)), sigma (list of (2,)), history) where
    history has 'cost', 'sigma_norm', 'x_trajs', 'sigmas' exactly as the reference fills them."""
    x_ref = np.asarray(x_ref, dtype=float)
    u_ref = np.asarray(u_ref, dtype=float)
    if u_ref.shape[0] == x_ref.shape[0]:
        if verbose:
            print(f" u_ref has same length as x_ref ({u_ref.shape[0]}). Using first N-1 controls.")
        u_ref = u_ref[:-1]
    if u_ref.shape[0] != x_ref.shape[0] - 1:
        raise ValueError(f"Incompatible dimensions: x_ref has {x_ref.shape[0]} states but u_ref has "
                         f"{u_ref.shape[0]} controls (expected {x_ref.shape[0]-1})")
    eng = _eng()
    solver = BatchedNewtonSolver(eng, x_ref, u_ref, 1, tol=tol, beta=beta, c=c, gamma_0=gamma_0,
                                 max_ls=MAX_LINE_SEARCH_ITERS, pipeline=False)
    x0 = np.asarray(x0, dtype=float).reshape(1, 4)
    solver.init(x0)
    solver.stream_sigma()   # one four-wavefront launch per iteration, sigma1 stored by its sweep (the same bits)
    Tn = x_ref.shape[0] - 1

    def lane_x(buf):
        return eng.unpack(solver.states(buf), 1)[0].cpu().numpy()

    x_traj = lane_x(0)
    assert x_traj.shape[0] == x_ref.shape[0], \
        f"Simulated trajectory length mismatch: {x_traj.shape[0]} vs {x_ref.shape[0]}"
    cost_k = float(solver.cost[0].item())
    history = {"cost": [cost_k], "sigma_norm": [], "x_trajs": [x_traj.copy()], "sigmas": []}
    trial_gammas = armijo_steps(gamma_0, beta, MAX_LINE_SEARCH_ITERS)
    for k in range(max_iters):
        prev_cost = cost_k
        plot = (k < plot_armijo_iters and (k % 2 == 0 or k < 3)) or k == 1000    # :372-381
        if plot:   # the trials' costs, bit for bit, and the pre-update iterate for the report
            trial_costs = solver.gamma_sweep(trial_gammas)[0].cpu().numpy()
            x_prev, u_prev = history["x_trajs"][-1], solver.controls(k & 1)[0].cpu().numpy()
            rolls = int(solver.n_roll[0].item())
        solver.iteration()
        # one device -> host copy per iteration: status, max|sigma|, cost, sigma (T,2) and the new iterate (N,4)
        rec = torch.cat([solver.status[:1].to(torch.float64), solver.smax[:1], solver.cost[:1],
                         solver.sigma()[0].reshape(-1),
                         eng.unpack(solver.states(solver.k & 1), 1)[0].reshape(-1)]).cpu().numpy()
        status = int(rec[0])
        sig = rec[3:3 + 2 * Tn].reshape(Tn, 2)
        history["sigmas"].append(list(sig))          # row views of this iteration's own (T,2) array
        history["sigma_norm"].append(float(rec[1]))
        if status == _lib.LS_FAILED:
            if verbose:
                print(f"Iteration {k}: Line search failed to find sufficient decrease.")
            break
        if plot:
            n_tested = int(solver.n_roll[0].item()) - rolls
            Kk = solver.gains()[0].cpu().numpy()
            plot_armijo_line_search(k, x_prev, u_prev, [Kk[t] for t in range(Tn)], [sig[t] for t in range(Tn)],
                                    prev_cost, x_ref, u_ref, float(solver.dJ[0].item()),
                                    float(solver.gamma[0].item()), list(trial_gammas[:n_tested]),
                                    list(trial_costs[:n_tested]), c, beta)
        cost_k = float(rec[2])
        history["cost"].append(cost_k)
        history["x_trajs"].append(rec[3 + 2 * Tn:].reshape(-1, 4))
        if verbose and k % 10 == 0:
            print(f"Iter {k}: Cost={cost_k:.2f}, diff_cost={prev_cost - cost_k:.2e}, ")
        if status == _lib.CONVERGED:
            if verbose:
                print(f"Converged at iteration {k}!")
            break
    x, u, K, s = solver.finalize()
    K = K[0].cpu().numpy(); s = s[0].cpu().numpy()
    return (x[0].cpu().numpy(), u[0].cpu().numpy(), [K[t] for t in range(Tn)], [s[t] for t in range(Tn)], history)


def newton_Algorithm_batch(x0, x_ref, u_ref, max_iters, tol=1e-6, beta=0.7, c=0.5, gamma_0=1.0,
                           max_ls=MAX_LINE_SEARCH_ITERS, hist_len=0, reduce_stats=None,
                           capture_lanes=None) -> SolveResult:
    """Batched newton_Algorithm over lanes x0 (B,4) sharing (x_ref, u_ref) -- or each with its own, x_ref (B,N,4) and
    u_ref (B,N-1 or N,2) -- -> SolveResult (device tensors).
    ``hist_len`` keeps every lane's cost / max|sigma| history; ``capture_lanes`` keeps the listed lanes'
    trajectories after every accepted iteration (SolveResult.x_trajs, the reference's history['x_trajs'])."""
    return newton_solve_batch(x0, x_ref, u_ref, max_iters, tol=tol, beta=beta, c=c, gamma_0=gamma_0, max_ls=max_ls,
                              engine=_eng(), hist_len=hist_len, reduce_stats=reduce_stats,
                              capture_lanes=capture_lanes)


def lane_history(res: SolveResult, lane: int) -> dict:
    """The reference's ``history`` dict (:321-327) of one lane of a batched solve, for generate_report_graphs:
    cost and sigma_norm from the per-lane histories (hist_len), x_trajs from capture_lanes.  'sigmas' has the
    reference's length (one entry per iteration the lane ran, :341) and holds sigma (T,2) at the iterations the
    report plots -- the solver's capture_sigma iterations (0, 1, 2 by default) and the last one (the solve's sigma
    output) -- and None at the others (the batched solver does not keep every iteration's sigma)."""
    if res.hist_cost is None or res.x_trajs is None or lane not in res.x_trajs:
        raise ValueError("lane_history needs a solve with hist_len > 0 and the lane in capture_lanes")
    n = int(res.n_iter[lane])
    failed = int(res.status[lane]) == _lib.LS_FAILED
    hc = res.hist_cost[:, lane].cpu().numpy()
    hs = res.hist_smax[:, lane].cpu().numpy()
    sigmas = [None] * n
    for it, sg in (res.sigmas or {}).get(lane, {}).items():
        if it < n:
            sigmas[it] = np.asarray(sg)
    if n:
        sigmas[n - 1] = res.sigma[lane].cpu().numpy()
    return {"cost": [res.cost0[lane]] + [float(v) for v in hc[:n - 1 if failed else n]],
            "sigma_norm": [float(v) for v in hs[:n]], "x_trajs": res.x_trajs[lane], "sigmas": sigmas}
