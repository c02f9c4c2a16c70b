"""CPU ORACLE (test infrastructure only) -- NumPy restatement of the reference's LQR / MPC trackers.

Only tests/ and bench.py's cpu_baseline leg may import this module; the product never does.

Restates /root/reference/trajectory_tracking.py (study of the source text; nothing copied):
  compute_P_inf        :144-165   fixed-point iteration of the discrete Riccati map until max|dP| < tol
  solve_LQR_tracking   :170-203   linearise along (x_opt, u_opt), backward recursion
                                  K = -inv(R + B'PB) B'PA,  P = Q + A'PA + (A'PB) K
  simulate_tracking    :206-216   u = u_opt + K (x - x_opt), x+ = RK4(x, u)
  solve_mpc_tracking   :8-69      receding horizon over a sliding window of the reference with (A_f, B_f)
                                  padding, T_pred = 75 (:10), Q = diag(120,100,1e-4,1e-4), R = diag(1e-6,10),
                                  Q_T = P_inf at x_f = [pi,0,0,0] (:31-38)
  solver_mpc           :73-140    the IPOPT QP.  It has only equality constraints (test_constraints = False,
                                  :87), so its solution is the finite-horizon LQ solution; here it is solved
                                  EXACTLY by a dense KKT system (mpc_qp_kkt) -- IPOPT itself (casadi) is not
                                  available, so parity with IPOPT's own iterates is unpinned (its tol is 1e-6).
Pinning: tests/test_tracking.py checks compute_P_inf / solve_LQR_tracking / simulate_tracking against
tests/golden/tracking.npz, produced by running the reference's own functions (make_golden_tracking.py).
"""
from __future__ import annotations

import numpy as np

from . import acrobot_np as ref

DT = ref.DT
Q_REG = np.diag([100.0, 100.0, 10.0, 10.0])        # trajectory_tracking.py:173
R_REG = np.diag([1.0, 1.0])                         # :174
QT_REG = Q_REG * 2.0                                # :175
Q_MPC = np.diag([120.0, 100.0, 0.0001, 0.0001])     # :36
R_MPC = np.diag([1e-6, 10.0])                       # :37
X_F = np.array([np.pi, 0.0, 0.0, 0.0])              # :31
U_F = np.array([0.0, 0.0])                          # :32
T_PRED = 75                                         # :10


def linearize_along(x_ref, u_ref, dt=DT):
    """A_d (S,4,4), B_d (S,4,2) at (x_ref[t], u_ref[t]), t < S = len(u_ref)  (:177-183, :17-25)."""
    S = u_ref.shape[0]
    A_c, B_c = ref.jacobians(x_ref[:S], u_ref[:S])
    return ref.discretize(A_c, B_c, dt)


def riccati_step(A, B, P, Q, R):
    aux1 = R + B.T @ P @ B
    aux2 = B.T @ P @ A
    K = -np.linalg.inv(aux1) @ aux2
    return K, Q + (A.T @ P @ A) + (A.T @ P @ B) @ K


def compute_P_inf(A, B, Q, R, max_iter=1000, tol=1e-6):
    """:144-165 (returns P and the iteration count, max_iter + 1 if the tolerance was never met: the reference
    then prints 'P_inf did not converge!!!', :164)."""
    P = Q
    for i in range(max_iter):
        P_prev = P
        _, P = riccati_step(A, B, P, Q, R)
        if np.abs(P - P_prev).max() < tol:
            return P, i + 1
    return P, max_iter + 1


def solve_LQR_tracking(x_opt, u_opt, Q=Q_REG, R=R_REG, QT=QT_REG):
    """:170-203 -> K (N-1, 2, 4)."""
    A, B = linearize_along(x_opt, u_opt)
    P = QT.copy()
    K = np.zeros((A.shape[0], 2, 4))
    for t in reversed(range(A.shape[0])):
        K[t], P = riccati_step(A[t], B[t], P, Q, R)
    return K


def simulate_tracking(x_opt, u_opt, K, x0):
    """:206-216 for a batch of initial states x0 (B,4) -> x (B,N,4), u (B,N-1,2)."""
    x0 = np.atleast_2d(np.asarray(x0, dtype=float))
    Bn, N = x0.shape[0], x_opt.shape[0]
    x = np.zeros((Bn, N, 4)); u = np.zeros((Bn, N - 1, 2))
    x[:, 0] = x0
    for t in range(N - 1):
        u[:, t] = u_opt[t] + np.einsum("ij,bj->bi", K[t], x[:, t] - x_opt[t])
        x[:, t + 1] = ref.rk4(x[:, t], u[:, t])
    return x, u


def mpc_windows(A, B, A_f, B_f, T_pred, n_steps):
    """The (A_list[:T_pred], B_list[:T_pred]) of control step t after t window shifts (:58-66)."""
    S = A.shape[0]
    for t in range(n_steps):
        idx = np.arange(t, t + T_pred)
        Aw = np.where((idx < S)[:, None, None], A[np.minimum(idx, S - 1)], A_f)
        Bw = np.where((idx < S)[:, None, None], B[np.minimum(idx, S - 1)], B_f)
        yield Aw, Bw


def mpc_first_gain(Aw, Bw, Q, R, QT):
    """First feedback gain of the window's LQ problem: stages 0..T_pred-2, terminal cost at T_pred-1."""
    P = QT
    K = None
    for s in reversed(range(Aw.shape[0] - 1)):
        K, P = riccati_step(Aw[s], Bw[s], P, Q, R)
    return K


def mpc_qp_kkt(x0, Aw, Bw, Q, R, QT):
    """Dense KKT solve of solver_mpc's QP (:73-140): variables X (T_pred,4), U (T_pred,2) minus the unused
    U[T_pred-1]; equalities X0 = x0 and X[t+1] = A_t X[t] + B_t U[t].  Returns (U0, X, U)."""
    Tp = Aw.shape[0]
    nxv, nuv = 4 * Tp, 2 * (Tp - 1)
    n = nxv + nuv
    H = np.zeros((n, n))
    for t in range(Tp - 1):
        H[4 * t:4 * t + 4, 4 * t:4 * t + 4] = 2 * Q
        H[nxv + 2 * t:nxv + 2 * t + 2, nxv + 2 * t:nxv + 2 * t + 2] = 2 * R
    H[4 * (Tp - 1):4 * Tp, 4 * (Tp - 1):4 * Tp] = 2 * QT
    m = 4 + 4 * (Tp - 1)
    E = np.zeros((m, n)); e = np.zeros(m)
    E[:4, :4] = np.eye(4); e[:4] = x0
    for t in range(Tp - 1):
        r = 4 + 4 * t
        E[r:r + 4, 4 * (t + 1):4 * (t + 2)] = np.eye(4)
        E[r:r + 4, 4 * t:4 * t + 4] = -Aw[t]
        E[r:r + 4, nxv + 2 * t:nxv + 2 * t + 2] = -Bw[t]
    KKT = np.block([[H, E.T], [E, np.zeros((m, m))]])
    sol = np.linalg.solve(KKT, np.concatenate([np.zeros(n), e]))
    X = sol[:nxv].reshape(Tp, 4); U = sol[nxv:n].reshape(Tp - 1, 2)
    return U[0], X, U


def mpc_gains(x_ref, u_ref, T_pred=T_PRED, Q=Q_MPC, R=R_MPC):
    """K0(t) (T-1, 2, 4) of every control step, and P_inf (:8-69 with the QP solved exactly)."""
    A, B = linearize_along(x_ref, u_ref)
    A_f, B_f = ref.discretize(*ref.jacobians(X_F[None], U_F[None]))
    A_f, B_f = A_f[0], B_f[0]
    QT, _ = compute_P_inf(A_f, B_f, Q, R)
    n_steps = x_ref.shape[0] - 1
    K0 = np.array([mpc_first_gain(Aw, Bw, Q, R, QT) for Aw, Bw in mpc_windows(A, B, A_f, B_f, T_pred, n_steps)])
    return K0, QT


def solve_mpc_tracking(x0, x_ref, u_ref, T_pred=T_PRED):
    """:8-69 for a batch x0 (B,4): x_real (B,N,4), u_real (B,N-1,2), K0 (N-1,2,4).
    u_real[t] = u_ref[t] + K0(t) (x_real[t] - x_ref[t]); x_real[t+1] = RK4(x_real[t], u_real[t])."""
    K0, _ = mpc_gains(x_ref, u_ref, T_pred)
    x, u = simulate_tracking(x_ref, u_ref, K0, x0)
    return x, u, K0
