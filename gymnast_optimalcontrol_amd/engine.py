"""Batched tensor-level front end of the HIP engine (device tensors in, device tensors out).

Every method is a thin launcher over one C-ABI entry point of include/gymnast_acrobot.h; the
arithmetic runs in the gfx950 kernels of csrc/acrobot_kernels.hip.  Inputs are fp64 tensors
(any device / numpy are copied to the engine's HIP device); outputs stay on the device.

Lane-major shapes follow the reference stacked over lanes: x (B,N,4), u (B,T,2), K (B,T,2,4),
sigma (B,T,2).  Internally trajectories live in the SoA "pairs" layout (see the header).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .params import PARAM_SETS, DT, Q_DIAG, R_DIAG, QT_DIAG

F64 = torch.float64


def padded(B: int) -> int:
    return max(64, (B + 63) // 64 * 64)


@dataclass
class Weights:
    Q: tuple = Q_DIAG
    R: tuple = R_DIAG
    QT: tuple = QT_DIAG

    def require_gain_solvable(self):
        """Checked wherever G is inverted (the solver, the gain sweeps; cost-only paths accept any weights, as the
        reference does).  R > 0: the reference's G = R_t + B^T P B is diag(2 R0, .) with B[:, 0] = 0, and
        np.linalg.solve raises on a singular G (trajectory_generation.py:203-204); the kernels divide by 2 R0 and
        2 R1 + b^T P b.  Q, Q_T >= 0: keeps every P positive semi-definite, so G11 = 2 R1 + b^T P b >= 2 R1 > 0 and
        1/G11 is in the range the kernels' reciprocal (rcp + two Newton steps, no IEEE range scaling) covers."""
        if not all(np.isfinite(v) and v > 0 for v in self.R):
            raise ValueError(f"R must be positive (G = diag(2 R0, 2 R1 + b^T P b) is inverted), got {self.R}")
        for name, v in (("Q", self.Q), ("Q_T", self.QT)):
            if not all(np.isfinite(x) and x >= 0 for x in v):
                raise ValueError(f"{name} must be non-negative for the gain sweeps (P stays PSD), got {v}")
        return self

    def c_struct(self) -> _lib.GymWeights:
        w = _lib.GymWeights()
        w.Q[:] = [float(v) for v in self.Q]
        w.R[:] = [float(v) for v in self.R]
        w.QT[:] = [float(v) for v in self.QT]
        return w

    @staticmethod
    def from_matrices(Q, R, QT) -> "Weights":
        """Diagonal weights from the reference's matrices; raises if they are not diagonal."""
        out = []
        for name, M, n in (("Q", Q, 4), ("R", R, 2), ("Q_T", QT, 4)):
            M = np.asarray(M, dtype=float)
            if M.shape != (n, n):
                raise ValueError(f"{name} must be {n}x{n}, got {M.shape}")
            if np.any(M - np.diag(np.diag(M))):
                raise NotImplementedError(f"the fused solver kernels take diagonal {name}; use the generic path")
            out.append(tuple(np.diag(M)))
        return Weights(*out)


class AcrobotEngine:
    """Launchers for one acrobot parameter set on one HIP device."""

    def __init__(self, params=1, dt: float = DT, weights: Weights | None = None, device=None,
                 lib_path: str = _lib.LIB_PATH):
        self.device = _lib.require_device(device, lib_path)
        self.lib = _lib.load(lib_path)
        p = PARAM_SETS[params] if isinstance(params, int) else params
        self.params = dict(p)
        self.dt = float(dt)
        self.model = _lib.GymModel()
        vec = np.array([p[k] for k in ("m1", "m2", "l1", "lc1", "l2", "lc2", "I1", "I2", "g", "f1", "f2")], float)
        _lib.check(self.lib.gym_model_from_params(vec.ctypes.data, self.dt, C.byref(self.model)),
                   "gym_model_from_params")
        self.weights = weights or Weights()
        self._w = self.weights.c_struct()

    # -------------------------------------------------------------------------------- utils
    def t(self, a, shape=None) -> torch.Tensor:
        """fp64 contiguous tensor on the engine device."""
        if isinstance(a, torch.Tensor):
            out = a.to(device=self.device, dtype=F64)
        else:
            out = torch.as_tensor(np.asarray(a, dtype=np.float64), device=self.device)
        if shape is not None:
            out = out.reshape(shape)
        return out.contiguous()

    @property
    def stream(self) -> int:
        return _lib.stream_handle(self.device)

    def set_weights(self, weights: Weights):
        w = weights.c_struct()          # first: a failure leaves the engine's weights unchanged
        self.weights, self._w = weights, w

    def pack(self, a: torch.Tensor, Bp: int, W: int = 2) -> torch.Tensor:
        """(B,L,C) lane-major -> SoA (L, C/W, Bp, W): W = 2 pairs (states, gains; wave-blocked, see the ABI header),
        W = 1 planes (controls, sigma).  The tensor shape only sizes the buffer: pair elements are laid out as
        (L, Bp/64, C/W, 64, 2)."""
        B, L, Cc = a.shape
        out = torch.empty((L, Cc // W, Bp, W), dtype=F64, device=self.device)
        _lib.check(self.lib.gym_pack_lanes(a.data_ptr(), out.data_ptr(), B, Bp, L, Cc, W, self.stream),
                   "gym_pack_lanes")
        return out

    def unpack(self, soa: torch.Tensor, B: int, soa1: torch.Tensor | None = None,
               sel: torch.Tensor | None = None) -> torch.Tensor:
        """SoA (L, P, Bp, W) -> lane-major (B, L, P*W); lane b reads soa1 where sel[b] != 0."""
        L, P, Bp, W = soa.shape
        out = torch.empty((B, L, P * W), dtype=F64, device=self.device)
        _lib.check(self.lib.gym_unpack_lanes(soa.data_ptr(), _lib.ptr(soa1), _lib.ptr(sel), out.data_ptr(), B, Bp,
                                             L, P * W, W, self.stream), "gym_unpack_lanes")
        return out

    def refs(self, x_ref, u_ref, per_lane: bool = False):
        """(x_ref (N,4), u_ref (N-1,2)) on the device, u_ref trimmed / checked as newton_Algorithm does; with
        ``per_lane`` also (B,N,4) / (B,N-1 or N,2) per-lane references (the batched solver, every schedule)."""
        x_ref = self.t(x_ref)
        u_ref = self.t(u_ref)
        lane = per_lane and x_ref.ndim == 3
        if (x_ref.ndim != (3 if lane else 2)) or x_ref.shape[-1] != 4:
            raise ValueError(f"x_ref must be (N,4){' or (B,N,4)' if per_lane else ''}, got {tuple(x_ref.shape)}")
        if u_ref.ndim != x_ref.ndim or u_ref.shape[-1] != 2 or (lane and u_ref.shape[0] != x_ref.shape[0]):
            raise ValueError(f"u_ref {tuple(u_ref.shape)} does not match x_ref {tuple(x_ref.shape)}")
        if u_ref.shape[-2] == x_ref.shape[-2]:      # trajectory_generation.py:301-303
            u_ref = u_ref[..., :-1, :].contiguous()
        if u_ref.shape[-2] != x_ref.shape[-2] - 1:
            raise ValueError(f"Incompatible dimensions: x_ref has {x_ref.shape[-2]} states but u_ref has "
                             f"{u_ref.shape[-2]} controls (expected {x_ref.shape[-2] - 1})")
        return x_ref.contiguous(), u_ref.contiguous()

    # --------------------------------------------------------------------- point primitives
    def _points(self, x, u):
        x = self.t(x); u = self.t(u)
        n = x.numel() // 4
        return x.reshape(n, 4), u.reshape(n, 2), n

    def continuous_dynamics(self, x, u) -> torch.Tensor:
        x, u, n = self._points(x, u)
        out = torch.empty((n, 4), dtype=F64, device=self.device)
        _lib.check(self.lib.gym_continuous_dynamics(C.byref(self.model), x.data_ptr(), u.data_ptr(), out.data_ptr(),
                                                    n, self.stream), "gym_continuous_dynamics")
        return out

    def rk4(self, x, u) -> torch.Tensor:
        x, u, n = self._points(x, u)
        out = torch.empty((n, 4), dtype=F64, device=self.device)
        _lib.check(self.lib.gym_rk4_step(C.byref(self.model), x.data_ptr(), u.data_ptr(), out.data_ptr(), n,
                                         self.stream), "gym_rk4_step")
        return out

    def jacobians(self, x, u):
        x, u, n = self._points(x, u)
        A = torch.empty((n, 4, 4), dtype=F64, device=self.device)
        Bm = torch.empty((n, 4, 2), dtype=F64, device=self.device)
        _lib.check(self.lib.gym_jacobians(C.byref(self.model), x.data_ptr(), u.data_ptr(), A.data_ptr(),
                                          Bm.data_ptr(), n, self.stream), "gym_jacobians")
        return A, Bm

    def stage_cost_derivs(self, x, x_ref, u, u_ref, Q, R, terminal=False):
        x = self.t(x).reshape(-1, 4); xr = self.t(x_ref).reshape(-1, 4)
        n = x.shape[0]
        Qm = np.ascontiguousarray(np.asarray(Q, float).reshape(4, 4))
        l = torch.empty(n, dtype=F64, device=self.device)
        gx = torch.empty((n, 4), dtype=F64, device=self.device)
        if terminal:
            u_ = ur_ = gu = None
            Rm = None
        else:
            u_ = self.t(u).reshape(-1, 2); ur_ = self.t(u_ref).reshape(-1, 2)
            Rm = np.ascontiguousarray(np.asarray(R, float).reshape(2, 2))
            gu = torch.empty((n, 2), dtype=F64, device=self.device)
        _lib.check(self.lib.gym_stage_cost_derivs(
            x.data_ptr(), xr.data_ptr(), _lib.ptr(u_), _lib.ptr(ur_), Qm.ctypes.data,
            None if Rm is None else Rm.ctypes.data, int(bool(terminal)), l.data_ptr(), gx.data_ptr(), _lib.ptr(gu),
            n, self.stream), "gym_stage_cost_derivs")
        return l, gx, gu

    # ----------------------------------------------------------------- trajectory kernels
    def rollout_open_loop(self, x0, u, x_ref, u_ref):
        """simulate_open_loop (+ total_cost): x0 (B,4), u (B,T,2) -> x (B,N,4), J (B,)."""
        x0 = self.t(x0).reshape(-1, 4)
        B = x0.shape[0]
        x_ref, u_ref = self.refs(x_ref, u_ref)
        N = x_ref.shape[0]
        u = self.t(u)
        if u.ndim == 2:
            u = u.expand(B, -1, -1).contiguous()
        if u.shape != (B, N - 1, 2):
            raise ValueError(f"u must be ({B},{N - 1},2), got {tuple(u.shape)}")
        Bp = padded(B)
        us = self.pack(u, Bp, W=1)
        xs = torch.empty((N, 2, Bp, 2), dtype=F64, device=self.device)
        J = torch.empty(Bp, dtype=F64, device=self.device)
        _lib.check(self.lib.gym_rollout_open_loop(C.byref(self.model), C.byref(self._w), x0.data_ptr(),
                                                  us.data_ptr(), x_ref.data_ptr(), u_ref.data_ptr(), xs.data_ptr(),
                                                  J.data_ptr(), B, Bp, N, self.stream), "gym_rollout_open_loop")
        return self.unpack(xs, B), J[:B]

    def closed_loop(self, x, u, K, sigma, gamma, x_ref, u_ref):
        """forward_closed_loop_update (+ total_cost of the result), full gains K (B,T,2,4)."""
        x = self.t(x); u = self.t(u); K = self.t(K); sigma = self.t(sigma)
        B, N, _ = x.shape
        T = N - 1
        x_ref, u_ref = self.refs(x_ref, u_ref)
        Bp = padded(B)
        g = torch.zeros(Bp, dtype=F64, device=self.device)
        g[:B] = self.t(gamma).reshape(-1).expand(B) if self.t(gamma).numel() == 1 else self.t(gamma).reshape(B)
        xs, us = self.pack(x, Bp), self.pack(u, Bp, W=1)
        Ks = self.pack(K.reshape(B, T, 8), Bp)
        ss = self.pack(sigma, Bp, W=1)
        xn = torch.empty_like(xs); un = torch.empty_like(us)
        J = torch.empty(Bp, dtype=F64, device=self.device)
        _lib.check(self.lib.gym_closed_loop(C.byref(self.model), C.byref(self._w), xs.data_ptr(), us.data_ptr(),
                                            Ks.data_ptr(), ss.data_ptr(), g.data_ptr(), x_ref.data_ptr(),
                                            u_ref.data_ptr(), xn.data_ptr(), un.data_ptr(), J.data_ptr(), B, Bp, N,
                                            self.stream), "gym_closed_loop")
        return self.unpack(xn, B), self.unpack(un, B), J[:B]

    def gamma_sweep(self, x, u, K, sigma, gammas, x_ref, u_ref) -> torch.Tensor:
        """J(gamma_g) of forward_closed_loop_update + total_cost for each lane and step size (the reference's
        Armijo line-search curve, plot_armijo_line_search :258-264): x (B,N,4), u (B,T,2), K (B,T,2,4),
        sigma (B,T,2), gammas (G,) -> (B, G)."""
        x = self.t(x); u = self.t(u); K = self.t(K); sigma = self.t(sigma)
        g = self.t(gammas).reshape(-1)
        B, N, _ = x.shape
        T = N - 1
        G = int(g.numel())
        if G < 1:
            raise ValueError("gamma_sweep needs at least one step size")
        x_ref, u_ref = self.refs(x_ref, u_ref)
        Bp = padded(B)
        xs, us = self.pack(x, Bp), self.pack(u, Bp, W=1)
        Ks = self.pack(K.reshape(B, T, 8), Bp)
        ss = self.pack(sigma, Bp, W=1)
        J = torch.empty((G, Bp), dtype=F64, device=self.device)
        _lib.check(self.lib.gym_gamma_sweep(C.byref(self.model), C.byref(self._w), xs.data_ptr(), us.data_ptr(),
                                            Ks.data_ptr(), ss.data_ptr(), g.data_ptr(), G, x_ref.data_ptr(),
                                            u_ref.data_ptr(), J.data_ptr(), B, Bp, N, self.stream), "gym_gamma_sweep")
        return J[:, :B].t()

    def total_cost(self, x, u, x_ref, u_ref, Q, R, QT):
        x = self.t(x); u = self.t(u)
        B, N, _ = x.shape
        x_ref = self.t(x_ref); u_ref = self.t(u_ref)[: N - 1].contiguous()
        Bp = padded(B)
        xs, us = self.pack(x, Bp), self.pack(u, Bp, W=1)
        mats = [np.ascontiguousarray(np.asarray(M, float)) for M in (Q, R, QT)]
        J = torch.empty(Bp, dtype=F64, device=self.device)
        _lib.check(self.lib.gym_total_cost(xs.data_ptr(), us.data_ptr(), x_ref.data_ptr(), u_ref.data_ptr(),
                                           mats[0].ctypes.data, mats[1].ctypes.data, mats[2].ctypes.data,
                                           J.data_ptr(), B, Bp, N, self.stream), "gym_total_cost")
        return J[:B]

    def backward(self, x, u, x_ref, u_ref, want_lambda=False, check_gains=True):
        """Fused costate + stage lists + Riccati: K (B,T,2,4), sigma (B,T,2), dJ (B,), max|sigma| (B,), lambda.
        ``check_gains=False``: the caller uses only lambda (compute_costate_trajectory), which needs no G^-1."""
        if check_gains:
            self.weights.require_gain_solvable()
        x = self.t(x); u = self.t(u)
        B, N, _ = x.shape
        T = N - 1
        x_ref, u_ref = self.refs(x_ref, u_ref)
        Bp = padded(B)
        xs, us = self.pack(x, Bp), self.pack(u, Bp, W=1)
        K1 = torch.empty((T, 2, Bp, 2), dtype=F64, device=self.device)
        sg = torch.empty((T, 2, Bp, 1), dtype=F64, device=self.device)
        dJ = torch.empty(Bp, dtype=F64, device=self.device)
        sm = torch.empty(Bp, dtype=F64, device=self.device)
        lam = torch.empty((N, 2, Bp, 2), dtype=F64, device=self.device) if want_lambda else None
        _lib.check(self.lib.gym_backward_sweep(C.byref(self.model), C.byref(self._w), xs.data_ptr(), us.data_ptr(),
                                               x_ref.data_ptr(), u_ref.data_ptr(), K1.data_ptr(), sg.data_ptr(),
                                               dJ.data_ptr(), sm.data_ptr(), _lib.ptr(lam), B, Bp, N, self.stream),
                   "gym_backward_sweep")
        K = torch.empty((B, T, 2, 4), dtype=F64, device=self.device)
        _lib.check(self.lib.gym_unpack_gains(K1.data_ptr(), K.data_ptr(), B, Bp, T, self.stream), "gym_unpack_gains")
        return K, self.unpack(sg, B), dJ[:B], sm[:B], (self.unpack(lam, B) if want_lambda else None)

    def linearize(self, x, u, x_ref, u_ref):
        """build_stage_lists: A_d (B,T,4,4), B_d (B,T,4,2), q (B,T,4), r (B,T,2), q_T (B,4)."""
        x = self.t(x); u = self.t(u)
        B, N, _ = x.shape
        T = N - 1
        x_ref, u_ref = self.refs(x_ref, u_ref)
        Bp = padded(B)
        xs, us = self.pack(x, Bp), self.pack(u, Bp, W=1)
        e = lambda *s: torch.empty(s, dtype=F64, device=self.device)  # noqa: E731
        Ad, Bd, q, r, qT = e(T, 16, Bp), e(T, 8, Bp), e(T, 4, Bp), e(T, 2, Bp), e(4, Bp)
        _lib.check(self.lib.gym_linearize(C.byref(self.model), C.byref(self._w), xs.data_ptr(), us.data_ptr(),
                                          x_ref.data_ptr(), u_ref.data_ptr(), Ad.data_ptr(), Bd.data_ptr(),
                                          q.data_ptr(), r.data_ptr(), qT.data_ptr(), B, Bp, N, self.stream),
                   "gym_linearize")
        lm = lambda a, *s: a[..., :B].permute(-1, *range(a.ndim - 1)).reshape(B, *s)  # noqa: E731
        return lm(Ad, T, 4, 4), lm(Bd, T, 4, 2), lm(q, T, 4), lm(r, T, 2), lm(qT, 4)

    def riccati_general(self, A, Bm, Q, R, S, q, r, QT, qT):
        """calculate_K_and_sigma on dense per-lane stage data (lane-major, broadcastable over lanes/time)."""
        A = self.t(A)
        B, T = A.shape[:2]
        Bp = padded(B)

        def soa(a, shape_tail):  # (B,T,*tail) or broadcastable -> (T, prod(tail), Bp)
            a = self.t(a).expand(B, T, *shape_tail) if a is not None else None
            n = int(np.prod(shape_tail))
            out = torch.zeros((T, n, Bp), dtype=F64, device=self.device)
            out[:, :, :B] = a.reshape(B, T, n).permute(1, 2, 0)
            return out

        def soa_t(a, shape_tail):
            a = self.t(a).expand(B, *shape_tail)
            n = int(np.prod(shape_tail))
            out = torch.zeros((n, Bp), dtype=F64, device=self.device)
            out[:, :B] = a.reshape(B, n).T
            return out

        As, Bs, Qs, Rs, Ss = soa(A, (4, 4)), soa(Bm, (4, 2)), soa(Q, (4, 4)), soa(R, (2, 2)), soa(S, (2, 4))
        qs, rs, QTs, qTs = soa(q, (4,)), soa(r, (2,)), soa_t(QT, (4, 4)), soa_t(qT, (4,))
        K = torch.empty((T, 8, Bp), dtype=F64, device=self.device)
        sg = torch.empty((T, 2, Bp), dtype=F64, device=self.device)
        dJ = torch.empty(Bp, dtype=F64, device=self.device)
        _lib.check(self.lib.gym_riccati_general(As.data_ptr(), Bs.data_ptr(), Qs.data_ptr(), Rs.data_ptr(),
                                                Ss.data_ptr(), qs.data_ptr(), rs.data_ptr(), QTs.data_ptr(),
                                                qTs.data_ptr(), K.data_ptr(), sg.data_ptr(), dJ.data_ptr(), B, Bp, T,
                                                self.stream), "gym_riccati_general")
        return (K[..., :B].permute(2, 0, 1).reshape(B, T, 2, 4), sg[..., :B].permute(2, 0, 1).contiguous(),
                dJ[:B])

    # ------------------------------------------------------------------ LQR / MPC trackers
    @staticmethod
    def _host_mat(M, n, name):
        M = np.ascontiguousarray(np.asarray(M, dtype=np.float64))
        if M.shape != (n, n):
            raise ValueError(f"{name} must be {n}x{n}, got {M.shape}")
        return M

    def tv_lqr_gains(self, A, Bm, Q, R, QT, L: int, nwin: int = 1, all_gains: bool = True, A_pad=None,
                     B_pad=None, discretize: bool = False) -> torch.Tensor:
        """Windowed time-varying LQR gains (gym_tv_lqr_gains): stages A (S,4,4), B (S,4,2) on the device.
        all_gains: (L-1,2,4) gains of window 0; else (nwin,2,4) first gains of windows 0..nwin-1."""
        A = self.t(A).reshape(-1, 4, 4); Bm = self.t(Bm).reshape(-1, 4, 2)
        S = A.shape[0]
        Ap = None if A_pad is None else self.t(A_pad).reshape(4, 4)
        Bp_ = None if B_pad is None else self.t(B_pad).reshape(4, 2)
        Qh, Rh = self._host_mat(Q, 4, "Q"), self._host_mat(R, 2, "R")
        QTd = self.t(QT).reshape(4, 4)                 # device: e.g. dare_fixed_point's P, no host round trip
        out = torch.empty(((L - 1) if all_gains else nwin, 2, 4), dtype=F64, device=self.device)
        _lib.check(self.lib.gym_tv_lqr_gains(A.data_ptr(), Bm.data_ptr(), S, _lib.ptr(Ap), _lib.ptr(Bp_),
                                             Qh.ctypes.data, Rh.ctypes.data, QTd.data_ptr(), int(L), int(nwin),
                                             int(bool(all_gains)), int(bool(discretize)), self.dt, out.data_ptr(),
                                             self.stream), "gym_tv_lqr_gains")
        return out

    def dare_fixed_point(self, A, Bm, Q, R, max_iter: int = 1000, tol: float = 1e-6):
        """compute_P_inf on the device: returns (P (4,4), iterations (1,) int32), both device tensors (no sync)."""
        A = self.t(A).reshape(4, 4); Bm = self.t(Bm).reshape(4, 2)
        Qh, Rh = self._host_mat(Q, 4, "Q"), self._host_mat(R, 2, "R")
        P = torch.empty((4, 4), dtype=F64, device=self.device)
        it = torch.zeros(1, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.gym_dare_fixed_point(A.data_ptr(), Bm.data_ptr(), Qh.ctypes.data, Rh.ctypes.data,
                                                 int(max_iter), float(tol), P.data_ptr(), it.data_ptr(), self.stream),
                   "gym_dare_fixed_point")
        return P, it

    def mpc_gains(self, x_ref, u_ref, x_f, u_f, Q, R, L: int, nwin: int, max_iter: int = 1000, tol: float = 1e-6):
        """Fused MPC gains (gym_mpc_gains): stage linearisations of (x_ref, u_ref) and of the pad (x_f, u_f),
        Q_T = compute_P_inf(A_f, B_f, Q, R), and each window's first gain.  Returns device tensors
        (K0 (nwin,2,4), Q_T (4,4), iterations (1,) int32); no host synchronisation."""
        x_ref = self.t(x_ref).reshape(-1, 4); u_ref = self.t(u_ref).reshape(-1, 2)
        x_f = self.t(x_f).reshape(4); u_f = self.t(u_f).reshape(2)
        S = x_ref.shape[0] - 1
        if u_ref.shape[0] < S:
            raise ValueError(f"u_ref must hold {S} stages, got {u_ref.shape[0]}")
        Qh, Rh = self._host_mat(Q, 4, "Q"), self._host_mat(R, 2, "R")
        K = torch.empty((nwin, 2, 4), dtype=F64, device=self.device)
        P = torch.empty((4, 4), dtype=F64, device=self.device)
        it = torch.zeros(1, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.gym_mpc_gains(C.byref(self.model), x_ref.data_ptr(), u_ref.data_ptr(), S, x_f.data_ptr(),
                                          u_f.data_ptr(), Qh.ctypes.data, Rh.ctypes.data, int(L), int(nwin),
                                          int(max_iter), float(tol), K.data_ptr(), P.data_ptr(), it.data_ptr(),
                                          self.stream), "gym_mpc_gains")
        return K, P, it

    def lq_forward(self, A, Bm, K, x0, L: int, A_pad=None, B_pad=None, discretize: bool = False):
        """One window's LQ forward pass: X (L,4), U (L-1,2)."""
        A = self.t(A).reshape(-1, 4, 4); Bm = self.t(Bm).reshape(-1, 4, 2)
        Ap = None if A_pad is None else self.t(A_pad).reshape(4, 4)
        Bp_ = None if B_pad is None else self.t(B_pad).reshape(4, 2)
        K = self.t(K).reshape(-1, 2, 4); x0 = self.t(x0).reshape(4)
        X = torch.empty((L, 4), dtype=F64, device=self.device)
        U = torch.empty((L - 1, 2), dtype=F64, device=self.device)
        _lib.check(self.lib.gym_lq_forward(A.data_ptr(), Bm.data_ptr(), A.shape[0], _lib.ptr(Ap), _lib.ptr(Bp_),
                                           int(bool(discretize)), self.dt, K.data_ptr(), x0.data_ptr(), int(L),
                                           X.data_ptr(), U.data_ptr(), self.stream), "gym_lq_forward")
        return X, U

    def track_rollout(self, x0, x_ff, u_ff, K, single: bool = False):
        """Batched closed-loop tracking: x0 (B,4) -> x (B,N,4), u (B,T,2) under the shared (x_ff, u_ff, K).
        single: one lane per trajectory instead of a lane pair (bit-identical; measurement / tests)."""
        x0 = self.t(x0).reshape(-1, 4)
        x_ff = self.t(x_ff).reshape(-1, 4); u_ff = self.t(u_ff).reshape(-1, 2); K = self.t(K).reshape(-1, 2, 4)
        N = x_ff.shape[0]
        if u_ff.shape[0] != N - 1 or K.shape[0] != N - 1:
            raise ValueError(f"feed-forward / gains must hold {N - 1} stages, got {u_ff.shape[0]} / {K.shape[0]}")
        B = x0.shape[0]
        x = torch.empty((B, N, 4), dtype=F64, device=self.device)
        u = torch.empty((B, N - 1, 2), dtype=F64, device=self.device)
        _lib.check(self.lib.gym_track_rollout_ex(C.byref(self.model), x0.data_ptr(), x_ff.data_ptr(),
                                                 u_ff.data_ptr(), K.data_ptr(), B, N,
                                                 _lib.TRACK_SINGLE if single else 0, x.data_ptr(), u.data_ptr(),
                                                 self.stream), "gym_track_rollout_ex")
        return x, u
