"""Drop-in for the reference's ``trajectory_tracking`` module (LQR and receding-horizon MPC trackers).

Reference: /root/reference/trajectory_tracking.py (main.py task_3 / task_4).  Same names, arguments and
return values; the arithmetic runs in the gfx950 kernels of csrc/tracking_kernels.hip (gym_tv_lqr_gains,
gym_dare_fixed_point, gym_lq_forward, gym_track_rollout) and the acrobot kernels (Jacobians, RK4).

The MPC QP (solver_mpc :73-140) has only equality constraints (test_constraints = False, :87), so its
solution is the finite-horizon LQ solution over the window; it is computed exactly (no IPOPT iterations):
u0 = K_0(t) x0 with K_0(t) the window's first gain.  Every lane follows the same reference, so the gains of
all T control steps are computed once (one window per thread) and the B perturbed initial states are then
simulated in closed loop in one batched kernel -- the same controls the per-step re-solve produces.

Batched additions: ``LQR_tracking_batch`` and ``solve_mpc_tracking_batch`` take x0 (B,4) and return device
tensors.  There is no CPU fallback.
"""
from __future__ import annotations

import numpy as np
import torch

from . import dynamics as _dyn
from .dynamics import dt, ns, ni  # noqa: F401  (the reference module's namespace, trajectory_tracking.py:3)

nu = ni
Q_REG = np.diag([100.0, 100.0, 10.0, 10.0])        # trajectory_tracking.py:173
R_REG = np.diag([1.0, 1.0])                         # :174
QT_REG = Q_REG * 2.0                                # :175
Q_MPC = np.diag([120.0, 100.0, 0.0001, 0.0001])     # :36
R_MPC = np.diag([1e-6, 10.0])                       # :37
X_F = np.array([np.pi, 0.0, 0.0, 0.0])              # :31
U_F = np.array([0.0, 0.0])                          # :32
T_PRED = 75                                         # :10
MPC_FUSED_MAX_STAGES = 256                          # gym_mpc_gains: T_pred + 2 stages per workgroup's LDS table


def _eng():
    return _dyn.engine()


def _np(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy()


_FINAL_STATE = {}


def _final_state(eng):
    """X_F, U_F (:31-32) as device tensors, made once per device: a pageable host-to-device copy inside every
    mpc_gains call would make the host wait for the GPU and leave the GPU idle while Python enqueues the run."""
    key = str(eng.device)
    if key not in _FINAL_STATE:
        _FINAL_STATE[key] = (eng.t(X_F.reshape(1, 4)), eng.t(U_F.reshape(1, 2)))
    return _FINAL_STATE[key]


def _discrete(eng, A_c, B_c):
    eye = torch.eye(4, dtype=A_c.dtype, device=A_c.device)
    return eye + eng.dt * A_c, eng.dt * B_c                      # trajectory_generation.py:161-164


def compute_P_inf(A, B, Q, R):
    """trajectory_tracking.py:144-165 (fixed-point iteration, max 1000 iterations, tol 1e-6)."""
    eng = _eng()
    P, it = eng.dare_fixed_point(A, B, Q, R, max_iter=1000, tol=1e-6)
    P = _np(P)
    if int(it.item()) > 1000:                    # the tolerance was never met in 1000 iterations (:164)
        print("P_inf did not converge!!!")
    return P


def solve_LQR_tracking(x_opt, u_opt):
    """trajectory_tracking.py:170-203 -> list of N-1 gains (2,4)."""
    K = lqr_gains(x_opt, u_opt)
    return list(_np(K))


def lqr_gains(x_opt, u_opt, Q=Q_REG, R=R_REG, QT=QT_REG) -> torch.Tensor:
    """Device form of solve_LQR_tracking: (N-1, 2, 4) tensor."""
    eng = _eng()
    x_opt = eng.t(x_opt).reshape(-1, 4)
    u_opt = eng.t(u_opt).reshape(-1, 2)
    S = x_opt.shape[0] - 1
    A_c, B_c = eng.jacobians(x_opt[:S], u_opt[:S])
    return eng.tv_lqr_gains(A_c, B_c, Q, R, QT, L=S + 1, nwin=1, all_gains=True, discretize=True)


def simulate_tracking(x_opt, u_opt, K_reg, x0_perturbed):
    """trajectory_tracking.py:206-216 -> (x_track (N,4), u_track (N-1,2)) numpy."""
    eng = _eng()
    K = eng.t(np.asarray([np.asarray(k, dtype=float) for k in K_reg]) if isinstance(K_reg, (list, tuple)) else K_reg)
    x, u = eng.track_rollout(np.asarray(x0_perturbed, dtype=float).reshape(1, 4), x_opt, u_opt, K)
    return _np(x[0]), _np(u[0])


def LQR_tracking(x_ref, u_ref, t_ref, x0_perturbed=None):
    """trajectory_tracking.py:219-249 (plotting omitted) -> (x_track, u_track)."""
    if x0_perturbed is None:
        x0_perturbed = np.asarray(x_ref)[0].copy()
    K_reg_seq = solve_LQR_tracking(x_ref, u_ref)
    return simulate_tracking(x_ref, u_ref, K_reg_seq, x0_perturbed)


def LQR_tracking_batch(x_ref, u_ref, x0):
    """Batched LQR tracking: x0 (B,4) -> (x (B,N,4), u (B,N-1,2), K (N-1,2,4)) device tensors."""
    eng = _eng()
    K = lqr_gains(x_ref, u_ref)
    x, u = eng.track_rollout(x0, x_ref, u_ref, K)
    return x, u, K


def mpc_gains(x_ref, u_ref, T_pred: int = T_PRED, Q=Q_MPC, R=R_MPC, n_steps: int | None = None):
    """K_0(t) (n_steps, 2, 4) of every control step of solve_mpc_tracking, and Q_T = P_inf (:8-69)."""
    eng = _eng()
    x_ref = eng.t(x_ref).reshape(-1, 4)
    u_ref = eng.t(u_ref).reshape(-1, 2)
    S = x_ref.shape[0] - 1                                          # A_list: one stage per u_ref row (:19)
    n_steps = S if n_steps is None else int(n_steps)
    x_f, u_f = _final_state(eng)
    if int(T_pred) + 2 <= MPC_FUSED_MAX_STAGES:
        # one launch: stage linearisations, compute_P_inf and every window's recursion (gym_mpc_gains)
        K0, QT, _ = eng.mpc_gains(x_ref, u_ref, x_f, u_f, Q, R, L=int(T_pred), nwin=n_steps)
        return K0, QT
    A_c, B_c = eng.jacobians(x_ref[:S], u_ref[:S])
    Af_c, Bf_c = eng.jacobians(x_f, u_f)
    A_f, B_f = _discrete(eng, Af_c[0], Bf_c[0])
    QT, _ = eng.dare_fixed_point(A_f, B_f, Q, R)
    K0 = eng.tv_lqr_gains(A_c, B_c, Q, R, QT, L=int(T_pred), nwin=n_steps, all_gains=False,
                          A_pad=Af_c[0], B_pad=Bf_c[0], discretize=True)
    return K0, QT


def solve_mpc_tracking_batch(x0, x_ref, u_ref, T_pred: int = T_PRED):
    """Batched receding-horizon MPC: x0 (B,4) -> (x_real (B,N,4), u_real (B,N-1,2), K0 (N-1,2,4))."""
    eng = _eng()
    K0, _ = mpc_gains(x_ref, u_ref, T_pred)
    x, u = eng.track_rollout(x0, x_ref, u_ref, K0)
    return x, u, K0


def solve_mpc_tracking(x0, x_ref, u_ref, T, T_pred: int = T_PRED):
    """trajectory_tracking.py:8-69 -> (x_real (N,4), u_real (N-1,2)); control steps t < T-1."""
    x_ref = np.asarray(x_ref, dtype=float)
    u_ref = np.asarray(u_ref, dtype=float)
    steps = int(T) - 1
    x_real = np.zeros(x_ref.shape)
    u_real = np.zeros(u_ref.shape)
    x, u, _ = solve_mpc_tracking_batch(np.asarray(x0, dtype=float).reshape(1, 4), x_ref, u_ref, T_pred)
    x_real[:steps + 1] = _np(x[0])[:steps + 1]
    u_real[:steps] = _np(u[0])[:steps]
    return x_real, u_real


def solver_mpc(x0, A_list, B_list, Q, R, Q_T, T_pred, u_ref=None):
    """trajectory_tracking.py:73-140: the window's QP solved exactly -> (U0 (2,), X_opt (T_pred,4),
    U_opt (T_pred,2)); U_opt's last row (no cost, no constraint in the reference's QP) is 0."""
    eng = _eng()
    A = eng.t(np.asarray(A_list[:T_pred], dtype=float)).reshape(-1, 4, 4)
    B = eng.t(np.asarray(B_list[:T_pred], dtype=float)).reshape(-1, 4, 2)
    K = eng.tv_lqr_gains(A, B, Q, R, Q_T, L=int(T_pred), nwin=1, all_gains=True,
                         A_pad=A[-1], B_pad=B[-1], discretize=False)
    X, U = eng.lq_forward(A, B, K, np.asarray(x0, dtype=float).reshape(4), int(T_pred), A_pad=A[-1], B_pad=B[-1])
    U_opt = np.zeros((int(T_pred), 2))
    U_opt[:-1] = _np(U)
    return U_opt[0].copy(), _np(X), U_opt
