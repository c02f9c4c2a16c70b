"""CPU ORACLE (test infrastructure only) -- NumPy restatement of the reference hot path.

This module is a *checker*. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import it; the product package (gymnast_optimalcontrol_amd) never does.

It restates, vectorised over a leading batch ("lane") axis, the reference's algorithm in the
same *dense* form the reference uses, so that it is an independent check of the HIP kernels'
closed-form / structure-exploiting arithmetic:

  * the acrobot model is built symbolically (sympy) from the textbook M, C, G, F of
    /root/reference/dynamics.py:63-90 (parameter set params_1, dynamics.py:15-29), and the
    continuous Jacobians are taken symbolically exactly as dynamics.py:157-170 does;
  * ``continuous_dynamics`` solves M qdd = RHS with a batched np.linalg.solve
    (dynamics.py:197-213, tau1 forced to 0 at :205);
  * the Riccati recursion is the dense one of trajectory_generation.py:183-216, with a
    batched np.linalg.solve on the 2x2 G.

Parity pin: tests/test_oracle_golden.py checks this module against the reference's own
golden npz (acrobot_optimal_trajectory.npz) and the vectors produced by running the
reference in the build container (tests/golden/make_golden.py).

Shapes: x (B,N,4), u (B,T,2), K (B,T,2,4), sigma (B,T,2); refs (N,4)/(T,2) shared.
"""
from __future__ import annotations

import functools

import numpy as np

# ---- problem constants (dynamics.py:173-175, trajectory_generation.py:8-18) -------------------
DT = 2e-2
NX, NU = 4, 2
T_HORIZON = 10.0
N_KNOTS = int(T_HORIZON / DT) + 1          # trajectory_generation.py:9 -> 501
Q_DEFAULT = np.diag([130.0, 30.0, 0.0001, 0.0001])   # :16
R_DEFAULT = np.diag([1e-6, 1.5])                     # :17
QT_DEFAULT = np.diag([130, 130.0, 1.0, 1.0])         # :18

# parameter sets (dynamics.py:15-61): m1 m2 l1 lc1 l2 lc2 I1 I2 g f1 f2
PARAM_SETS = {
    1: dict(m1=1.0, m2=1.0, l1=1.0, lc1=0.5, l2=1.0, lc2=0.5, I1=0.33, I2=0.33, g=9.81, f1=1.0, f2=1.0),
    2: dict(m1=2.0, m2=2.0, l1=1.5, lc1=0.75, l2=1.5, lc2=0.75, I1=1.5, I2=1.5, g=9.81, f1=1.0, f2=1.0),
    3: dict(m1=1.5, m2=1.5, l1=2.0, lc1=1.0, l2=2.0, lc2=1.0, I1=2.0, I2=2.0, g=9.81, f1=1.0, f2=1.0),
}


@functools.lru_cache(maxsize=4)
def _model(pset: int = 1):
    """Symbolic acrobot model -> lambdified (M, RHS, A_c, B_c) for one parameter set.

    Follows dynamics.py:63-90 (M, C, G, F), :109-113 (RHS, M_func), :153-170 (tau=[0,tau2],
    f_cont=[qdot; M^-1 RHS], A=df/dx, B=df/du)."""
    import sympy as sp
    th1, th2, w1, w2, t1, t2 = sp.symbols("th1 th2 w1 w2 t1 t2")
    p = {k: sp.Float(v) for k, v in PARAM_SETS[pset].items()}
    m1, m2, l1, lc1, lc2, I1, I2, g, f1, f2 = (p[k] for k in ("m1", "m2", "l1", "lc1", "lc2", "I1", "I2", "g", "f1", "f2"))
    M = sp.Matrix([[I1 + I2 + lc1**2 * m1 + m2 * (l1**2 + 2 * l1 * lc2 * sp.cos(th2) + lc2**2),
                    I2 + lc2 * m2 * (l1 * sp.cos(th2) + lc2)],
                   [I2 + lc2 * m2 * (l1 * sp.cos(th2) + lc2), I2 + lc2**2 * m2]])
    C = sp.Matrix([[-l1 * lc2 * m2 * w2 * sp.sin(th2), -l1 * lc2 * m2 * (w1 + w2) * sp.sin(th2)],
                   [l1 * lc2 * m2 * w1 * sp.sin(th2), 0]])
    G = sp.Matrix([g * lc1 * m1 * sp.sin(th1) + g * m2 * (l1 * sp.sin(th1) + lc2 * sp.sin(th1 + th2)),
                   g * m2 * lc2 * sp.sin(th1 + th2)])
    F = sp.Matrix([[f1, 0], [0, f2]])
    qd = sp.Matrix([w1, w2])
    rhs = sp.Matrix([0, t2]) - ((C + F) * qd + G)        # acrobot: only the elbow is driven
    f = sp.Matrix.vstack(qd, M.LUsolve(rhs))
    xs, us = [th1, th2, w1, w2], [t1, t2]
    A = f.jacobian(xs)
    Bm = f.jacobian(us)
    args = xs + us
    return ([[sp.lambdify([th1, th2], M[i, j], "numpy") for j in range(2)] for i in range(2)],
            [sp.lambdify(args, rhs[i], "numpy") for i in range(2)],
            [[sp.lambdify(args, A[i, j], "numpy") for j in range(4)] for i in range(4)],
            [[sp.lambdify(args, Bm[i, j], "numpy") for j in range(2)] for i in range(4)])


def _bcast(v, n):
    return np.broadcast_to(np.asarray(v, dtype=float), (n,))


def continuous_dynamics(x, u, pset=1):
    """x (B,4), u (B,2) -> xdot (B,4).  dynamics.py:197-213 (np.linalg.solve on M)."""
    x = np.atleast_2d(np.asarray(x, float)); u = np.atleast_2d(np.asarray(u, float))
    n = x.shape[0]
    Mf, Rf, _, _ = _model(pset)
    M = np.stack([np.stack([_bcast(Mf[i][j](x[:, 0], x[:, 1]), n) for j in range(2)], -1) for i in range(2)], -2)
    args = (x[:, 0], x[:, 1], x[:, 2], x[:, 3], 0.0 * u[:, 0], u[:, 1])   # tau1 = 0 (dynamics.py:205)
    rhs = np.stack([_bcast(Rf[i](*args), n) for i in range(2)], -1)
    qdd = np.linalg.solve(M, rhs[..., None])[..., 0]
    return np.concatenate([x[:, 2:4], qdd], axis=1)


def rk4(x, u, dt=DT, pset=1):
    """Classic RK4 with u held (dynamics.py:177-195)."""
    k1 = continuous_dynamics(x, u, pset)
    k2 = continuous_dynamics(x + (dt / 2) * k1, u, pset)
    k3 = continuous_dynamics(x + (dt / 2) * k2, u, pset)
    k4 = continuous_dynamics(x + dt * k3, u, pset)
    return x + dt * (k1 + 2 * k2 + 2 * k3 + k4) / 6.0


def jacobians(x, u, pset=1):
    """Continuous A_c (B,4,4), B_c (B,4,2) (dynamics.py:217-226 via the symbolic Jacobians :163-164)."""
    x = np.atleast_2d(np.asarray(x, float)); u = np.atleast_2d(np.asarray(u, float))
    n = x.shape[0]
    _, _, Af, Bf = _model(pset)
    args = (x[:, 0], x[:, 1], x[:, 2], x[:, 3], u[:, 0], u[:, 1])
    A = np.stack([np.stack([_bcast(Af[i][j](*args), n) for j in range(4)], -1) for i in range(4)], -2)
    B = np.stack([np.stack([_bcast(Bf[i][j](*args), n) for j in range(2)], -1) for i in range(4)], -2)
    return A, B


def discretize(A_c, B_c, dt=DT):
    """Forward-Euler linearisation (trajectory_generation.py:161-164)."""
    return np.eye(A_c.shape[-1]) + dt * A_c, dt * B_c


# ---- trajectory-level primitives ---------------------------------------------------------------

def simulate_open_loop(x0, u, pset=1):
    """x0 (B,4), u (B,T,2) -> x (B,T+1,4)   (trajectory_generation.py:74-87)."""
    x0 = np.atleast_2d(x0); u = np.asarray(u, float)
    if u.ndim == 2:
        u = np.broadcast_to(u, (x0.shape[0],) + u.shape)
    T = u.shape[1]
    x = np.zeros((x0.shape[0], T + 1, 4)); x[:, 0] = x0
    for t in range(T):
        x[:, t + 1] = rk4(x[:, t], u[:, t], pset=pset)
    return x


def total_cost(x, u, x_ref, u_ref, Q=Q_DEFAULT, R=R_DEFAULT, QT=QT_DEFAULT):
    """Batched J (trajectory_generation.py:231-252): stage weights Q, R (not 2Q), terminal Q_T."""
    dx = x - x_ref; du = u - u_ref
    J = np.zeros(x.shape[0])
    for t in range(x.shape[1] - 1):
        J += np.einsum("bi,ij,bj->b", dx[:, t], Q, dx[:, t])
        J += np.einsum("bi,ij,bj->b", du[:, t], R, du[:, t])
    return J + np.einsum("bi,ij,bj->b", dx[:, -1], QT, dx[:, -1])


def costate(x, u, x_ref, u_ref, Q=Q_DEFAULT, QT=QT_DEFAULT, pset=1):
    """lambda (B,N,4): lambda_N = 2 Q_T dx_N; lambda_t = 2 Q dx_t + A_d^T lambda_{t+1} (:138-159)."""
    B, N = x.shape[:2]
    lam = np.zeros((B, N, 4))
    lam[:, -1] = (2 * QT @ (x[:, -1] - x_ref[-1]).T).T
    for t in range(N - 2, -1, -1):
        A_c, _ = jacobians(x[:, t], u[:, t], pset)
        A_d = np.eye(4) + A_c * DT
        lam[:, t] = (2 * Q @ (x[:, t] - x_ref[t]).T).T + np.einsum("bji,bj->bi", A_d, lam[:, t + 1])
    return lam


def stage_lists(x, u, x_ref, u_ref, Q=Q_DEFAULT, R=R_DEFAULT, QT=QT_DEFAULT, pset=1):
    """Dense LQ stage data (build_stage_lists, :166-181): A_d, B_d, q, r per stage + terminal."""
    B, N = x.shape[:2]
    T = N - 1
    A_d = np.zeros((B, T, 4, 4)); B_d = np.zeros((B, T, 4, 2))
    for t in range(T):
        A_c, B_c = jacobians(x[:, t], u[:, t], pset)
        A_d[:, t], B_d[:, t] = discretize(A_c, B_c)
    q = np.einsum("ij,btj->bti", 2 * Q, x[:, :T] - x_ref[:T])
    r = np.einsum("ij,btj->bti", 2 * R, u - u_ref)
    qT = np.einsum("ij,bj->bi", 2 * QT, x[:, -1] - x_ref[-1])
    return A_d, B_d, q, r, 2 * QT, qT


def riccati(A_d, B_d, Qs, Rs, Ss, q, r, QT_blk, qT):
    """Dense batched Riccati (calculate_K_and_sigma, :183-216).

    A_d (B,T,4,4), B_d (B,T,4,2), Qs (B,T,4,4)|(4,4), Rs (B,T,2,2)|(2,2), Ss (B,T,2,4)|(2,4),
    q (B,T,4), r (B,T,2), QT_blk (B,4,4)|(4,4), qT (B,4) -> K (B,T,2,4), sigma (B,T,2), dJ (B,)."""
    Bn, T = A_d.shape[:2]
    bc = lambda M, t: M[:, t] if M.ndim == 4 else M  # noqa: E731
    P = np.broadcast_to(QT_blk, (Bn, 4, 4)).copy()
    p = qT.copy()
    K = np.zeros((Bn, T, 2, 4)); sig = np.zeros((Bn, T, 2)); dJ = np.zeros(Bn)
    for t in range(T - 1, -1, -1):
        A = A_d[:, t]; Bm = B_d[:, t]
        Qt, Rt, St = bc(Qs, t), bc(Rs, t), bc(Ss, t)
        BT = np.swapaxes(Bm, 1, 2); AT = np.swapaxes(A, 1, 2)
        G = Rt + BT @ P @ Bm
        F = St + BT @ P @ A
        g = r[:, t] + np.einsum("bij,bj->bi", BT, p)
        Kt = -np.linalg.solve(G, F)
        st = -np.linalg.solve(G, g[..., None])[..., 0]
        dJ += np.einsum("bi,bi->b", g, st)
        KT = np.swapaxes(Kt, 1, 2)
        P = Qt + AT @ P @ A - KT @ G @ Kt
        p = q[:, t] + np.einsum("bij,bj->bi", AT, p) - np.einsum("bij,bj->bi", KT @ G, st)
        K[:, t] = Kt; sig[:, t] = st
    return K, sig, dJ


def closed_loop(x, u, K, sig, gamma, pset=1):
    """u_new = u + K (x_new - x) + gamma sigma; x_new = RK4 (forward_closed_loop_update, :218-229).

    gamma is a scalar or a per-lane (B,) array."""
    B, N = x.shape[:2]
    gamma = np.broadcast_to(np.asarray(gamma, float), (B,))
    xn = x.copy(); un = u.copy()
    for t in range(N - 1):
        dx = xn[:, t] - x[:, t]
        un[:, t] = u[:, t] + np.einsum("bij,bj->bi", K[:, t], dx) + gamma[:, None] * sig[:, t]
        xn[:, t + 1] = rk4(xn[:, t], un[:, t], pset=pset)
    return xn, un


def gamma_sweep(x, u, K, sig, gammas, x_ref, u_ref, Q=Q_DEFAULT, R=R_DEFAULT, QT=QT_DEFAULT, pset=1):
    """plot_armijo_line_search's curve (trajectory_generation.py:256-264): for one trajectory x (N,4),
    u (T,2), K (T,2,4), sigma (T,2), J(gamma) = total_cost(forward_closed_loop_update(..., gamma)) per
    step size -> (G,).  The G rollouts run as G lanes of closed_loop."""
    g = np.asarray(gammas, float).reshape(-1)
    G = g.shape[0]
    rep = lambda a: np.repeat(np.asarray(a, float)[None], G, axis=0)   # noqa: E731
    xn, un = closed_loop(rep(x), rep(u), rep(K), rep(sig), g, pset=pset)
    return total_cost(xn, un, x_ref, u_ref, Q, R, QT)


# ---- the Newton / Armijo driver -----------------------------------------------------------------
ACTIVE, CONVERGED, LS_FAILED, MAX_ITERS = 0, 1, 2, 3


class NewtonStepper:
    """One outer iteration of newton_Algorithm (trajectory_generation.py:329-396) per call, for every lane.

    Same per-lane semantics as the reference: u-ref trim (:301-306), u0 = 0 open-loop init (:311-312),
    Armijo with strict '<' (:361) and gamma *= beta (:365), LS failure -> stop without update (:367-369),
    update then stop on max|sigma| < tol (:383-396).  ``iteration()`` returns the 8 statistics the HIP
    solver reports (gymnast_optimalcontrol_amd.solver.STAT_FIELDS), so the multi-rank loop logic can be
    exercised on CPU with this oracle as the per-shard engine."""

    def __init__(self, x0, x_ref, u_ref, tol=1e-6, beta=0.7, c=0.5, gamma_0=1.0, max_ls=20,
                 Q=Q_DEFAULT, R=R_DEFAULT, QT=QT_DEFAULT, pset=1):
        x0 = np.atleast_2d(np.asarray(x0, float))
        u_ref = np.asarray(u_ref, float)
        if u_ref.shape[0] == x_ref.shape[0]:
            u_ref = u_ref[:-1]
        if u_ref.shape[0] != x_ref.shape[0] - 1:
            raise ValueError("Incompatible dimensions")
        self.x_ref, self.u_ref = np.asarray(x_ref, float), u_ref
        self.tol, self.beta, self.c, self.gamma_0, self.max_ls = tol, beta, c, gamma_0, max_ls
        self.Q, self.R, self.QT, self.pset = Q, R, QT, pset
        Bn = x0.shape[0]
        self.u = np.zeros((Bn,) + u_ref.shape)
        self.x = simulate_open_loop(x0, self.u, pset)
        self.J = total_cost(self.x, self.u, self.x_ref, u_ref, Q, R, QT)
        self.status = np.full(Bn, ACTIVE); self.n_iter = np.zeros(Bn, int); self.n_roll = np.zeros(Bn, int)
        self.K = np.zeros((Bn, u_ref.shape[0], 2, 4)); self.sig = np.zeros((Bn, u_ref.shape[0], 2))
        self.smax = np.zeros(Bn)
        self.cost_hist = [self.J.copy()]; self.signorm_hist = []
        self.k = 0

    def iteration(self):
        Q, R, QT, pset = self.Q, self.R, self.QT, self.pset
        x, u, J, Bn = self.x, self.u, self.J, self.x.shape[0]
        ia = np.nonzero(self.status == ACTIVE)[0]
        sn = np.full(Bn, np.nan); ch = np.full(Bn, np.nan)
        n_retry = 0
        if ia.size:
            A_d, B_d, q, r, QTb, qT = stage_lists(x[ia], u[ia], self.x_ref, self.u_ref, Q, R, QT, pset)
            Ka, sa, dJ = riccati(A_d, B_d, 2 * Q, 2 * R, np.zeros((2, 4)), q, r, QTb, qT)
            self.K[ia] = Ka; self.sig[ia] = sa
            smax = np.max(np.abs(sa), axis=(1, 2))
            self.smax[ia] = smax; sn[ia] = smax
            gam = np.full(ia.size, float(self.gamma_0))
            done = np.zeros(ia.size, bool); ok = np.zeros(ia.size, bool)
            xn_acc = x[ia].copy(); un_acc = u[ia].copy(); Jn_acc = J[ia].copy()
            for i in range(self.max_ls):
                todo = np.nonzero(~done)[0]
                if todo.size == 0:
                    break
                if i == 1:
                    n_retry = todo.size
                xn, un = closed_loop(x[ia[todo]], u[ia[todo]], Ka[todo], sa[todo], gam[todo], pset)
                Jn = total_cost(xn, un, self.x_ref, self.u_ref, Q, R, QT)
                self.n_roll[ia[todo]] += 1
                acc = Jn < J[ia[todo]] + self.c * gam[todo] * dJ[todo]
                sel = todo[acc]
                xn_acc[sel] = xn[acc]; un_acc[sel] = un[acc]; Jn_acc[sel] = Jn[acc]
                ok[sel] = True; done[sel] = True
                gam[todo[~acc]] *= self.beta
            self.n_iter[ia] += 1
            self.status[ia[~ok]] = LS_FAILED
            good = ia[ok]
            x[good] = xn_acc[ok]; u[good] = un_acc[ok]; J[good] = Jn_acc[ok]
            self.status[ia[ok & (smax < self.tol)]] = CONVERGED
            ch[good] = J[good]
        self.signorm_hist.append(sn); self.cost_hist.append(ch)
        ran = self.n_iter == self.k + 1
        self.k += 1
        return np.array([np.sum(self.status == ACTIVE), np.sum(J), np.sum(self.smax[ran] ** 2), np.sum(ran),
                         n_retry, np.sum(self.status == CONVERGED), np.sum(self.status == LS_FAILED),
                         np.sum(self.n_roll)], dtype=float)

    def result(self):
        status = self.status.copy()
        status[status == ACTIVE] = MAX_ITERS
        return dict(x=self.x, u=self.u, K=self.K, sigma=self.sig, n_iter=self.n_iter, status=status, cost=self.J,
                    n_rollouts=self.n_roll, cost_hist=np.array(self.cost_hist),
                    sigma_norm_hist=np.array(self.signorm_hist))


def newton_solve(x0, x_ref, u_ref, max_iters, tol=1e-6, beta=0.7, c=0.5, gamma_0=1.0, max_ls=20,
                 Q=Q_DEFAULT, R=R_DEFAULT, QT=QT_DEFAULT, pset=1):
    """Per-lane semantics of newton_Algorithm (trajectory_generation.py:298-398), vectorised over lanes."""
    st = NewtonStepper(x0, x_ref, u_ref, tol, beta, c, gamma_0, max_ls, Q, R, QT, pset)
    for _k in range(max_iters):
        if not (st.status == ACTIVE).any():
            break
        st.iteration()
    return st.result()


def load_task2_refs(path):
    """get_fully_actuated_ref (trajectory_generation.py:511-518): u_ref = 2*[0, u_fa[:,1]]."""
    d = np.load(path)
    u_ref = np.zeros(d["u"].shape)
    u_ref[:, 1] = d["u"][:, 1]
    return d["x"], np.multiply(u_ref, 2), d["time"]
