"""CPU ORACLE (test infrastructure only) -- ctypes wrapper around oracle/build/libacrobot_oracle.so.

The plain-C restatement (acrobot_oracle.c) is the fast checker for full Newton solves and the
CPU baseline timed by bench.py (``cpu_baseline.kind = "port"``).  Never imported by the product.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libacrobot_oracle.so")

PARAMS_1 = (1.0, 1.0, 1.0, 0.5, 1.0, 0.5, 0.33, 0.33, 9.81, 1.0, 1.0)   # dynamics.py:15-29


class Model(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("a", "b", "d", "g1", "g2", "f1", "f2", "dt")]


class Cost(C.Structure):
    _fields_ = [("Q", C.c_double * 4), ("R", C.c_double * 2), ("QT", C.c_double * 4)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        dp = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
        ip = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        L.orc_model_from_params.argtypes = [dp, C.c_double, C.POINTER(Model)]
        solve_args = [C.POINTER(Model), C.POINTER(Cost), dp, dp, dp, C.c_int64, C.c_int, C.c_int]
        L.orc_newton_solve.argtypes = solve_args + [C.c_double, C.c_double, C.c_double, C.c_double, C.c_int,
                                                    dp, dp, dp, dp, ip, ip, dp, ip]
        L.orc_newton_iters.argtypes = solve_args + [C.c_double, C.c_double, C.c_double, C.c_int,
                                                    dp, dp, dp, dp, ip, ip, dp, ip]
        L.orc_newton_solve_hist.argtypes = solve_args + [C.c_double, C.c_double, C.c_double, C.c_double, C.c_int,
                                                         dp, dp, dp, dp, ip, ip, dp, ip, C.c_int, dp, dp, ip, dp]
        L.orc_rk4.argtypes = [C.POINTER(Model), dp, dp, dp]
        L.orc_jac.argtypes = [C.POINTER(Model), dp, dp, dp, dp, dp]
        _lib = L
    return _lib


def model(params=PARAMS_1, dt=2e-2):
    m = Model()
    lib().orc_model_from_params(np.asarray(params, np.float64), dt, C.byref(m))
    return m


def cost(Q=(130.0, 30.0, 1e-4, 1e-4), R=(1e-6, 1.5), QT=(130.0, 130.0, 1.0, 1.0)):
    c = Cost()
    c.Q[:] = list(Q); c.R[:] = list(R); c.QT[:] = list(QT)
    return c


def newton_solve(x0, x_ref, u_ref, max_iters=5000, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20,
                 fixed_iters=None, params=PARAMS_1, weights=None, hist_len=0):
    """Batched solve on host cores (OpenMP). x0 (B,4). Returns dict like acrobot_np.newton_solve.

    hist_len > 0 adds the per-iteration record of every lane, (B, hist_len) arrays, NaN / 0 past a lane's last
    iteration: ``hist_cost`` (cost after iteration k; NaN for a failed iteration, as the GPU's history), ``hist_smax`` (max|sigma| of its
    sweep), ``hist_trials`` (Armijo trials evaluated) and ``hist_margin`` (the iteration's tightest Armijo test,
    min |J_new - (J + c gamma dJ)| / |J| over its trials: how close the closest accept / reject call was to a tie)."""
    x0 = np.ascontiguousarray(np.atleast_2d(x0), np.float64)
    x_ref = np.ascontiguousarray(x_ref, np.float64)
    u_ref = np.ascontiguousarray(u_ref, np.float64)
    if u_ref.shape[0] == x_ref.shape[0]:
        u_ref = np.ascontiguousarray(u_ref[:-1])
    B, N = x0.shape[0], x_ref.shape[0]
    T = N - 1
    out = dict(x=np.zeros((B, N, 4)), u=np.zeros((B, T, 2)), K1=np.zeros((B, T, 4)), sigma=np.zeros((B, T, 2)),
               n_iter=np.zeros(B, np.int32), status=np.zeros(B, np.int32), cost=np.zeros(B),
               n_rollouts=np.zeros(B, np.int32))
    m = model(params); cw = cost(**(weights or {}))
    tail = (out["x"], out["u"], out["K1"], out["sigma"], out["n_iter"], out["status"], out["cost"], out["n_rollouts"])
    if hist_len and fixed_iters is None:
        H = int(hist_len)
        for k in ("hist_cost", "hist_smax", "hist_margin"):
            out[k] = np.full((B, H), np.nan)
        out["hist_trials"] = np.zeros((B, H), np.int32)
        lib().orc_newton_solve_hist(C.byref(m), C.byref(cw), x0, x_ref, u_ref, B, N, max_iters, tol, beta, c,
                                    gamma_0, max_ls, *tail, H, out["hist_cost"], out["hist_smax"],
                                    out["hist_trials"], out["hist_margin"])
    elif fixed_iters is None:
        lib().orc_newton_solve(C.byref(m), C.byref(cw), x0, x_ref, u_ref, B, N, max_iters, tol, beta, c, gamma_0,
                               max_ls, *tail)
    else:
        lib().orc_newton_iters(C.byref(m), C.byref(cw), x0, x_ref, u_ref, B, N, int(fixed_iters), beta, c, gamma_0,
                               max_ls, *tail)
    K = np.zeros((B, T, 2, 4)); K[:, :, 1, :] = out["K1"]
    out["K"] = K
    return out


def rk4(x, u, params=PARAMS_1):
    x = np.ascontiguousarray(x, np.float64); u = np.ascontiguousarray(u, np.float64)
    xn = np.zeros(4)
    lib().orc_rk4(C.byref(model(params)), x, u, xn)
    return xn


def jacobians(x, u, params=PARAMS_1):
    """A_c (4,4), B_c (4,2) from the closed form."""
    a2 = np.zeros(4); a3 = np.zeros(4); bc = np.zeros(2)
    lib().orc_jac(C.byref(model(params)), np.ascontiguousarray(x, np.float64), np.ascontiguousarray(u, np.float64),
                  a2, a3, bc)
    A = np.zeros((4, 4)); A[0, 2] = 1; A[1, 3] = 1; A[2] = a2; A[3] = a3
    B = np.zeros((4, 2)); B[2, 1] = bc[0]; B[3, 1] = bc[1]
    return A, B
