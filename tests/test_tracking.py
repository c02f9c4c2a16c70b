"""LQR / receding-horizon MPC trackers (trajectory_tracking.py).

Golden data: tests/golden/tracking.npz, produced by running the reference's own compute_P_inf,
solve_LQR_tracking and simulate_tracking (tests/golden/make_golden_tracking.py).  The MPC's IPOPT QP
(solver_mpc) cannot run here (casadi is absent): MPC parity is pinned to the exact solution of that
equality-constrained QP (dense KKT solve in oracle/tracking_np.py), not to IPOPT's iterates.
Tolerances: gains 1e-9 relative (same recursion, reordered 4x4 products), closed-loop trajectories 1e-9
rel-L2.
"""
import numpy as np
import pytest

from conftest import load_golden, rel_l2

TOL = 1e-9


@pytest.fixture(scope="module")
def trk():
    return load_golden("tracking")


# ------------------------------------------------------------------------------ oracle (CPU)
def test_oracle_lqr_matches_reference_golden(trk):
    from oracle import tracking_np as tr
    K = tr.solve_LQR_tracking(trk["x_opt"], trk["u_opt"])
    assert np.abs(K - trk["K_reg"]).max() <= 1e-10 * np.abs(trk["K_reg"]).max()
    x, u = tr.simulate_tracking(trk["x_opt"], trk["u_opt"], trk["K_reg"], trk["x_opt"][0][None] + trk["dx"][:, None])
    assert rel_l2(x, trk["x_track"]) < 1e-12 and rel_l2(u, trk["u_track"]) < 1e-12


def test_oracle_p_inf_matches_reference_golden(trk):
    from oracle import tracking_np as tr
    P, it = tr.compute_P_inf(trk["A_f"], trk["B_f"], trk["Q_mpc"], trk["R_mpc"])
    np.testing.assert_array_equal(P, trk["P_inf"])
    # SURVEY.md 8(c) KAT: diag(P_inf) ~ [2.257e7, 1.674e6, 3.202e6, 3.610e5]
    np.testing.assert_allclose(np.diag(P), [2.257e7, 1.674e6, 3.202e6, 3.610e5], rtol=2e-3)


@pytest.mark.parametrize("t", [0, 137, 430, 499])
def test_oracle_mpc_gain_is_the_exact_qp_solution(trk, t):
    """u0 = K_0(t) x0 equals the dense KKT solution of solver_mpc's QP for the window of control step t."""
    from oracle import tracking_np as tr
    A, B = tr.linearize_along(trk["x_opt"], trk["u_opt"])
    QT, _ = tr.compute_P_inf(trk["A_f"], trk["B_f"], tr.Q_MPC, tr.R_MPC)
    for Tp in (50, 75):
        Aw, Bw = list(tr.mpc_windows(A, B, trk["A_f"], trk["B_f"], Tp, t + 1))[t]
        K0 = tr.mpc_first_gain(Aw, Bw, tr.Q_MPC, tr.R_MPC, QT)
        x0 = np.random.default_rng(t).uniform(-0.2, 0.2, 4)
        U0, X, U = tr.mpc_qp_kkt(x0, Aw, Bw, tr.Q_MPC, tr.R_MPC, QT)
        np.testing.assert_allclose(K0 @ x0, U0, rtol=1e-8, atol=1e-10 * max(1.0, np.abs(U0).max()))


# ------------------------------------------------------------------------------ HIP path
@pytest.mark.gpu
def test_lqr_gains_and_tracking_match_reference(trk):
    from gymnast_optimalcontrol_amd import trajectory_tracking as tt
    K = np.asarray(tt.solve_LQR_tracking(trk["x_opt"], trk["u_opt"]))
    assert K.shape == (500, 2, 4)
    assert np.abs(K - trk["K_reg"]).max() <= TOL * np.abs(trk["K_reg"]).max()
    for i, dx in enumerate(trk["dx"]):
        x, u = tt.LQR_tracking(trk["x_opt"], trk["u_opt"], trk["t_ref"], x0_perturbed=trk["x_opt"][0] + dx)
        assert rel_l2(x, trk["x_track"][i]) < TOL and rel_l2(u, trk["u_track"][i]) < TOL


@pytest.mark.gpu
def test_lqr_batch_equals_single_lane(trk):
    from gymnast_optimalcontrol_amd import trajectory_tracking as tt
    from oracle import tracking_np as tr
    B = 200
    x0 = trk["x_opt"][0] + np.random.default_rng(3).uniform(-0.3, 0.3, (B, 4))
    x, u, K = tt.LQR_tracking_batch(trk["x_opt"], trk["u_opt"], x0)
    xo, uo = tr.simulate_tracking(trk["x_opt"], trk["u_opt"], trk["K_reg"], x0)
    assert rel_l2(x.cpu().numpy(), xo) < TOL and rel_l2(u.cpu().numpy(), uo) < TOL
    xs, us = tt.simulate_tracking(trk["x_opt"], trk["u_opt"], list(K.cpu().numpy()), x0[7])   # same gains
    np.testing.assert_array_equal(xs, x[7].cpu().numpy())


@pytest.mark.gpu
def test_p_inf_on_device(trk):
    from gymnast_optimalcontrol_amd import trajectory_tracking as tt
    P = tt.compute_P_inf(trk["A_f"], trk["B_f"], trk["Q_mpc"], trk["R_mpc"])
    np.testing.assert_allclose(P, trk["P_inf"], rtol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("T_pred", [50, 75])
def test_mpc_gains_and_closed_loop_match_oracle(trk, T_pred):
    from gymnast_optimalcontrol_amd import trajectory_tracking as tt
    from oracle import tracking_np as tr
    K0, QT = tt.mpc_gains(trk["x_opt"], trk["u_opt"], T_pred)
    K0o, QTo = tr.mpc_gains(trk["x_opt"], trk["u_opt"], T_pred)
    np.testing.assert_allclose(QT.cpu().numpy(), QTo, rtol=1e-9)
    assert np.abs(K0.cpu().numpy() - K0o).max() <= TOL * np.abs(K0o).max()
    B = 65
    x0 = trk["x_opt"][0] + np.random.default_rng(T_pred).uniform(-0.1, 0.1, (B, 4))
    x0[0] = trk["x_opt"][0] + 0.1                       # main.task_4's disturbance
    x, u, _ = tt.solve_mpc_tracking_batch(x0, trk["x_opt"], trk["u_opt"], T_pred)
    xo, uo = tr.simulate_tracking(trk["x_opt"], trk["u_opt"], K0o, x0)
    assert rel_l2(x.cpu().numpy(), xo) < TOL and rel_l2(u.cpu().numpy(), uo) < TOL
    # reference-shaped entry point (task_4: T = len(t_ref))
    xr, ur = tt.solve_mpc_tracking(x0[0], trk["x_opt"], trk["u_opt"], len(trk["t_ref"]), T_pred=T_pred)
    assert xr.shape == trk["x_opt"].shape and ur.shape == trk["u_opt"].shape
    np.testing.assert_array_equal(xr, x[0].cpu().numpy())


@pytest.mark.gpu
def test_solver_mpc_window_matches_kkt(trk):
    from gymnast_optimalcontrol_amd import trajectory_tracking as tt
    from oracle import tracking_np as tr
    A, B = tr.linearize_along(trk["x_opt"], trk["u_opt"])
    QT, _ = tr.compute_P_inf(trk["A_f"], trk["B_f"], tr.Q_MPC, tr.R_MPC)
    Tp = 75
    Aw, Bw = A[100:100 + Tp], B[100:100 + Tp]
    x0 = np.array([0.05, -0.02, 0.1, 0.0])
    U0, X, U = tt.solver_mpc(x0, list(Aw), list(Bw), tr.Q_MPC, tr.R_MPC, QT, Tp)
    U0o, Xo, Uo = tr.mpc_qp_kkt(x0, Aw, Bw, tr.Q_MPC, tr.R_MPC, QT)
    np.testing.assert_allclose(U0, U0o, rtol=1e-8, atol=1e-12)
    assert X.shape == (Tp, 4) and U.shape == (Tp, 2)
    assert rel_l2(X, Xo) < 1e-8 and rel_l2(U[:-1], Uo) < 1e-8


@pytest.mark.gpu
def test_tracking_abi_rejects_bad_arguments():
    import ctypes as C
    from gymnast_optimalcontrol_amd import _lib
    lib = _lib.load()
    Q = np.eye(4); R = np.eye(2)
    # window past the end of the stages without a pad stage
    assert lib.gym_tv_lqr_gains(1, 1, 10, None, None, Q.ctypes.data, R.ctypes.data, Q.ctypes.data, 20, 1, 1, 0,
                                0.02, 1, None) == 1
    # all_gains needs a single window
    assert lib.gym_tv_lqr_gains(1, 1, 100, None, None, Q.ctypes.data, R.ctypes.data, Q.ctypes.data, 20, 2, 1, 0,
                                0.02, 1, None) == 1
    m = _lib.GymModel()
    assert lib.gym_track_rollout(C.byref(m), 1, 1, 1, 1, 0, 501, 1, 1, None) == 1          # empty batch
    assert lib.gym_track_rollout(C.byref(m), 1, 1, 1, 1, 100, 1, 1, 1, None) == 1          # N < 2


def _slow_pair():
    """(A, B) whose fixed point does not settle in 1000 iterations: the last two states are uncontrollable and
    marginally stable (A = I there), so P grows by Q each iteration -- finite, never within tol."""
    A = np.eye(4)
    A[0, 2] = A[1, 3] = 0.02
    B = np.zeros((4, 2)); B[0, 0] = B[1, 1] = 0.05
    return A, B


def test_oracle_p_inf_reports_non_convergence():
    from oracle import tracking_np as tr
    A, B = _slow_pair()
    P, it = tr.compute_P_inf(A, B, np.eye(4), np.eye(2))
    assert it == 1001 and np.isfinite(P).all()
    assert P[3, 3] > 1000.0                       # grows by at least Q_33 = 1 per iteration


@pytest.mark.gpu
def test_p_inf_prints_when_not_converged(capsys, trk):
    """The reference prints 'P_inf did not converge!!!' whenever the 1000-iteration loop ends without meeting
    the tolerance, and returns the (finite) last P (trajectory_tracking.py:164-165); on convergence it is
    silent."""
    from gymnast_optimalcontrol_amd import trajectory_tracking as tt
    from oracle import tracking_np as tr
    A, B = _slow_pair()
    P = tt.compute_P_inf(A, B, np.eye(4), np.eye(2))
    assert "P_inf did not converge!!!" in capsys.readouterr().out
    Po, _ = tr.compute_P_inf(A, B, np.eye(4), np.eye(2))
    np.testing.assert_allclose(P, Po, rtol=1e-12)
    tt.compute_P_inf(trk["A_f"], trk["B_f"], trk["Q_mpc"], trk["R_mpc"])
    assert "did not converge" not in capsys.readouterr().out


@pytest.mark.gpu
@pytest.mark.parametrize("T_pred", [2, 50, 75])
def test_fused_mpc_gains_match_the_generic_path(trk, T_pred):
    """gym_mpc_gains (stage linearisations, compute_P_inf and every window's recursion in one launch, lane-parallel
    structured Riccati map) against the generic kernels on host-built Jacobians (gym_jacobians,
    gym_dare_fixed_point, gym_tv_lqr_gains): gains and Q_T to 1e-11.

    The fused kernel computes Q_T = compute_P_inf with doubling jumps and then the reference's loop to its stop test;
    the generic kernel runs the reference's loop from P = Q.  On this pad the stop index is set by rounding: P[0][0]
    ~ 2.26e7 (ulp 3.7e-9) and max|dP| meanders around tol = 1e-6 for the last ~100 iterations (the reference stops at
    434 on its own A_f, the generic kernel at ~440 on the device's, the jump at ~517), all within ~4e-12 relative of
    each other."""
    from gymnast_optimalcontrol_amd import trajectory_tracking as tt
    eng = tt._eng()
    x_ref, u_ref = eng.t(trk["x_opt"]), eng.t(trk["u_opt"])
    S = x_ref.shape[0] - 1
    x_f, u_f = tt._final_state(eng)
    K0, QT, it = eng.mpc_gains(x_ref, u_ref, x_f, u_f, tt.Q_MPC, tt.R_MPC, L=T_pred, nwin=S)
    A_c, B_c = eng.jacobians(x_ref[:S], u_ref[:S])
    Af_c, Bf_c = eng.jacobians(x_f, u_f)
    A_f, B_f = tt._discrete(eng, Af_c[0], Bf_c[0])
    QTg, itg = eng.dare_fixed_point(A_f, B_f, tt.Q_MPC, tt.R_MPC)
    K0g = eng.tv_lqr_gains(A_c, B_c, tt.Q_MPC, tt.R_MPC, QTg, L=T_pred, nwin=S, all_gains=False,
                           A_pad=Af_c[0], B_pad=Bf_c[0], discretize=True)
    n, ng = int(it.item()), int(itg.item())
    assert 420 <= n <= 600 and 420 <= ng <= 460, (n, ng)  # the reference's count (converged); the reference's
    np.testing.assert_allclose(QT.cpu().numpy(), trk["P_inf"], rtol=1e-11)   # ... own P_inf (tracking.npz)
    np.testing.assert_allclose(QT.cpu().numpy(), QTg.cpu().numpy(), rtol=1e-11)
    Kg = K0g.cpu().numpy()
    assert np.abs(K0.cpu().numpy() - Kg).max() <= 1e-11 * np.abs(Kg).max()


@pytest.mark.gpu
@pytest.mark.parametrize("scale", [1e-2, 1e-4, 1e-6])
def test_fused_p_inf_stops_where_the_reference_stops(trk, scale):
    """Q_T must be the reference's stop iterate for any Q / R, not the DARE limit.  With Q, R scaled by
    1e-2 .. 1e-6 (P ~ 2e5 .. 23, tol = 1e-6 fixed) the limit lies 5e-11 .. 5e-7 relative beyond the reference's stop;
    the fused kernel (doubling jumps, then the reference's loop and test) must take the NumPy restatement's iteration
    count exactly and its P to rounding, and the generic fixed-point kernel likewise."""
    from gymnast_optimalcontrol_amd import trajectory_tracking as tt
    from oracle import tracking_np as tr
    eng = tt._eng()
    Q, R = np.asarray(tt.Q_MPC, float) * scale, np.asarray(tt.R_MPC, float) * scale
    x_ref, u_ref = eng.t(trk["x_opt"]), eng.t(trk["u_opt"])
    x_f, u_f = tt._final_state(eng)
    _, QT, it = eng.mpc_gains(x_ref, u_ref, x_f, u_f, Q, R, L=50, nwin=8)
    Po, ito = tr.compute_P_inf(trk["A_f"], trk["B_f"], Q, R)
    assert int(it.item()) == ito < 1000, (int(it.item()), ito)
    np.testing.assert_allclose(QT.cpu().numpy(), Po, rtol=1e-10, atol=1e-10 * np.abs(Po).max())
    Pg, itg = eng.dare_fixed_point(trk["A_f"], trk["B_f"], Q, R)
    assert int(itg.item()) == ito
    np.testing.assert_allclose(Pg.cpu().numpy(), Po, rtol=1e-10, atol=1e-10 * np.abs(Po).max())


@pytest.mark.gpu
def test_fused_mpc_gains_rejects_bad_arguments():
    import ctypes as C
    from gymnast_optimalcontrol_amd import _lib
    lib = _lib.load()
    m = _lib.GymModel()
    Q = np.eye(4); R = np.eye(2)
    args = lambda L, nwin, S=500: (C.byref(m), 1, 1, S, 1, 1, Q.ctypes.data, R.ctypes.data, L, nwin, 1000, 1e-6,
                                   1, 1, 1, None)
    assert lib.gym_mpc_gains(*args(1, 10)) == 1          # L < 2
    assert lib.gym_mpc_gains(*args(255, 10)) == 1        # L + 2 > 256 stages of the LDS table
    assert lib.gym_mpc_gains(*args(50, 0)) == 1          # no window
    assert lib.gym_mpc_gains(*args(50, 10, S=0)) == 1    # no stage


@pytest.mark.gpu
def test_pair_rollout_is_bitwise_the_single_lane_rollout(trk):
    """gym_track_rollout's default kernel (each trajectory on a lane pair, trigonometry split, DPP exchange)
    against the one-lane-per-trajectory kernel: identical bits, on a ragged batch that also holds lanes whose
    velocities take the sub-step full-reduction branch (|w| > 39 rad/s), a NaN lane and the MPC gains."""
    from gymnast_optimalcontrol_amd import trajectory_tracking as tt
    eng = tt._eng()
    B = 101
    rng = np.random.default_rng(11)
    x0 = trk["x_opt"][0] + rng.uniform(-0.1, 0.1, (B, 4))
    x0[3, 2:] = [45.0, -60.0]                            # sub-step angles beyond pi/4: full reductions
    x0[7, 0] = np.nan
    x0[9, :2] = [3.0e3, -2.0e3]                          # large angles
    K0, _ = tt.mpc_gains(trk["x_opt"], trk["u_opt"], 50)
    xp, up = eng.track_rollout(x0, trk["x_opt"], trk["u_opt"], K0)
    xs, us = eng.track_rollout(x0, trk["x_opt"], trk["u_opt"], K0, single=True)
    assert torch_equal_nan(xp, xs) and torch_equal_nan(up, us)
    assert np.isnan(xp[7, 1:].cpu().numpy()).all() and np.isfinite(xp[0].cpu().numpy()).all()


def torch_equal_nan(a, b):
    import torch
    return bool(torch.equal(torch.nan_to_num(a, nan=7.25), torch.nan_to_num(b, nan=7.25))) and \
        bool(torch.equal(torch.isnan(a), torch.isnan(b)))
