"""Parity of the HIP path (through the C-ABI) against the reference's golden vectors and the oracle.

Tolerances: the kernels use closed-form dynamics/Jacobians and a structure-exploiting Riccati,
i.e. the reference's arithmetic reordered, so per-primitive results agree to ~1e-12 relative and
converged trajectories to ~1e-13; the north-star bar for converged trajectories is 1e-8 rel-L2.
Discrete decisions (iteration counts, Armijo trials, statuses) must match exactly.
"""
import os
import sys

import numpy as np
import pytest

from conftest import rel_l2

pytestmark = pytest.mark.gpu

TOL_TRAJ = 1e-8        # north star: converged trajectory within 1e-8 relative L2


@pytest.fixture(scope="module")
def eng():
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    return AcrobotEngine()


@pytest.fixture(scope="module")
def tg():
    from gymnast_optimalcontrol_amd import trajectory_generation
    return trajectory_generation


def test_native_library_is_loaded(eng):
    import ctypes
    from gymnast_optimalcontrol_amd import _lib
    assert eng.lib._name == _lib.LIB_PATH
    assert ctypes.CDLL(_lib.LIB_PATH).gym_abi_version() == _lib.ABI_VERSION


# ------------------------------------------------------------------------------ primitives
def test_point_primitives_vs_reference(eng, golden):
    g = golden("kat_primitives")
    X, U = g["X"], g["U"]
    np.testing.assert_allclose(eng.continuous_dynamics(X, U).cpu().numpy(), g["f_cont"], rtol=1e-11, atol=1e-9)
    np.testing.assert_allclose(eng.rk4(X, U).cpu().numpy(), g["f_rk4"], rtol=1e-11, atol=1e-9)
    A, B = eng.jacobians(X, U)
    np.testing.assert_allclose(A.cpu().numpy(), g["A_c"], rtol=1e-10, atol=1e-8)
    np.testing.assert_allclose(B.cpu().numpy(), g["B_c"], rtol=1e-10, atol=1e-12)


def test_trigonometry_quadrants_and_domain(eng):
    """The device sin/cos (acrobot_device.hpp fast_sincos: Cody-Waite reduction, quadrant selects and sign bits)
    through gym_continuous_dynamics against the NumPy oracle (libm sin / cos): every quadrant, both signs, -0,
    angles at multiples of pi/2 and next to them, large arguments inside the domain; outside it (|th| * 2/pi >= 2^20,
    inf, NaN) the accelerations are NaN, so such a lane's cost is NaN and Armijo fails as for any non-finite value."""
    from oracle import acrobot_np as ref
    k = np.arange(-24, 25)
    base = np.concatenate([k * (np.pi / 2), k * (np.pi / 2) + 1e-9, k * (np.pi / 2) - 1e-9, k * 0.37 + 0.011,
                           [0.0, -0.0, 1e-300, -1e-300, 3.0, -3.0]])
    big = np.array([1e3, -1e3, 12345.678, -98765.4321, 1e5, -1e5, 1.6e6, -1.6e6])
    rng = np.random.default_rng(5)
    ang = np.concatenate([base, big])
    n = len(ang)
    X = np.stack([ang, rng.permutation(ang), rng.uniform(-3, 3, n), rng.uniform(-3, 3, n)], 1)
    U = np.stack([np.zeros(n), rng.uniform(-2, 2, n)], 1)
    got = eng.continuous_dynamics(X, U).cpu().numpy()
    want = ref.continuous_dynamics(X, U)
    small = (np.abs(X[:, 0]) < 100) & (np.abs(X[:, 1]) < 100)
    np.testing.assert_allclose(got[small], want[small], rtol=1e-12, atol=1e-12)
    # large in-domain arguments: the reduction's error grows with the quadrant count (2-term pi/2)
    np.testing.assert_allclose(got[~small], want[~small], rtol=1e-8, atol=1e-8)
    out = np.array([1.7e6, -1.7e6, 1e7, 1e300, np.inf, -np.inf, np.nan])
    m = len(out)
    Xo = np.stack([out, np.full(m, 0.3), np.zeros(m), np.zeros(m)], 1)
    Xo2 = np.stack([np.full(m, 0.3), out, np.zeros(m), np.zeros(m)], 1)
    Uo = np.zeros((m, 2))
    for Xd in (Xo, Xo2):
        g = eng.continuous_dynamics(Xd, Uo).cpu().numpy()
        assert np.isnan(g[:, 2:]).all(), g


def test_reference_style_point_calls(tg, golden):
    from gymnast_optimalcontrol_amd import dynamics as dyn
    g = golden("kat_primitives")
    for i in (0, 1, 2, 3, 4, 5, 17):
        np.testing.assert_allclose(dyn.dynamics(g["X"][i], g["U"][i]), g["f_rk4"][i], rtol=1e-11, atol=1e-9)
        np.testing.assert_allclose(dyn.continuous_dynamics(g["X"][i], g["U"][i]), g["f_cont"][i], rtol=1e-11,
                                   atol=1e-9)
        A, B = dyn.Calculate_A_B_matrixes(g["X"][i], g["U"][i])
        assert A.shape == (4, 4) and B.shape == (4, 2)
        np.testing.assert_allclose(A, g["A_c"][i], rtol=1e-10, atol=1e-8)
        Ad, Bd = tg.discretize_linearization(A, B, dyn.dt)
        np.testing.assert_allclose(Ad, g["A_d"][i], rtol=1e-10, atol=1e-10)
    # column-vector inputs are squeezed like the reference (dynamics.py:181-182)
    np.testing.assert_allclose(dyn.dynamics(g["X"][0][:, None], g["U"][0][:, None]), g["f_rk4"][0], rtol=1e-11)


def test_stage_cost_derivatives(tg, golden):
    g = golden("kat_primitives")
    for i in range(0, 64, 9):
        l, gx, gu, Hx, Hu = tg.derivatives_Cost(g["X"][i], g["xr"][i], g["U"][i], g["ur"][i], g["Qg"], g["Rg"])
        assert l == pytest.approx(float(g["l"][i]), rel=1e-12)
        np.testing.assert_allclose(gx, g["gx"][i], rtol=1e-12)
        np.testing.assert_allclose(gu, g["gu"][i], rtol=1e-12)
        np.testing.assert_array_equal(Hx, 2 * g["Qg"])
        lT, gT, HT = tg.derivatives_Cost(g["X"][i], g["xr"][i], g["U"][i], g["ur"][i], None, None, Q_T=g["QTg"],
                                         terminal=True)
        assert lT == pytest.approx(float(g["lT"][i]), rel=1e-12)
        np.testing.assert_allclose(gT, g["gT"][i], rtol=1e-12)


# ---------------------------------------------------------------------- one Newton iteration
@pytest.mark.parametrize("tag", ["it0", "mid"])
def test_newton_iteration_pieces(tg, golden, tag):
    g = golden("newton_iteration")
    x, u, xr, ur = g[f"{tag}_x"], g[f"{tag}_u"], g["x_ref"], g["u_ref"]
    lam = np.asarray(tg.compute_costate_trajectory(x, u, xr, ur))
    assert rel_l2(lam, g[f"{tag}_lambda"]) < 1e-12
    lists = tg.build_stage_lists(x, u, xr, ur, list(lam))
    np.testing.assert_allclose(np.asarray(lists[0]), g[f"{tag}_A_d"], rtol=1e-11, atol=1e-11)
    np.testing.assert_allclose(np.asarray(lists[1]), g[f"{tag}_B_d"], rtol=1e-11, atol=1e-14)
    np.testing.assert_allclose(np.asarray(lists[5]), g[f"{tag}_q"], rtol=1e-13)
    np.testing.assert_allclose(np.asarray(lists[6]), g[f"{tag}_r"], rtol=1e-13)
    np.testing.assert_allclose(lists[8], g[f"{tag}_qT"], rtol=1e-13)
    K, sig, dJ = tg.calculate_K_and_sigma(*lists)          # generic dense Riccati kernel
    assert rel_l2(np.asarray(K), g[f"{tag}_K"]) < 1e-10
    assert rel_l2(np.asarray(sig), g[f"{tag}_sigma"]) < 1e-10
    assert dJ == pytest.approx(float(g[f"{tag}_dJ"]), rel=1e-10)
    for gam, sfx in ((0.1, "01"), (1.0, "1")):
        xn, un = tg.forward_closed_loop_update(x, u, g[f"{tag}_K"], g[f"{tag}_sigma"], gamma=gam)
        assert rel_l2(xn, g[f"{tag}_xn{sfx}"]) < 1e-10
        assert rel_l2(un, g[f"{tag}_un{sfx}"]) < 1e-10
        J = tg.total_cost(xn, un, xr, ur, tg.Q, tg.R, tg.Q_T)
        assert J == pytest.approx(float(g[f"{tag}_cost{sfx}"]), rel=1e-11)
    assert tg.total_cost(x, u, xr, ur, tg.Q, tg.R, tg.Q_T) == pytest.approx(float(g[f"{tag}_cost"]), rel=1e-13)


@pytest.mark.parametrize("tag", ["it0", "mid"])
def test_fused_backward_sweep(eng, golden, tag):
    """The solver's fused structured sweep equals the reference's dense K, sigma, dJ, max|sigma|."""
    g = golden("newton_iteration")
    K, sig, dJ, smax, lam = eng.backward(g[f"{tag}_x"][None], g[f"{tag}_u"][None], g["x_ref"], g["u_ref"],
                                         want_lambda=True)
    assert rel_l2(K[0].cpu().numpy(), g[f"{tag}_K"]) < 1e-10
    assert rel_l2(sig[0].cpu().numpy(), g[f"{tag}_sigma"]) < 1e-10
    assert float(dJ[0]) == pytest.approx(float(g[f"{tag}_dJ"]), rel=1e-10)
    assert float(smax[0]) == pytest.approx(np.abs(g[f"{tag}_sigma"]).max(), rel=1e-10)
    assert rel_l2(lam[0].cpu().numpy(), g[f"{tag}_lambda"]) < 1e-12
    assert np.all(K[0, :, 0, :].cpu().numpy() == 0)


def test_general_riccati(tg, golden):
    g = golden("newton_iteration")
    K, sig, dJ = tg.calculate_K_and_sigma(list(g["gen_A"]), list(g["gen_B"]), list(g["gen_Q"]), list(g["gen_R"]),
                                          list(g["gen_S"]), list(g["gen_q"]), list(g["gen_r"]), g["gen_QT"],
                                          g["gen_qT"])
    assert rel_l2(np.asarray(K), g["gen_K"]) < 1e-12
    assert rel_l2(np.asarray(sig), g["gen_sigma"]) < 1e-12
    assert dJ == pytest.approx(float(g["gen_dJ"]), rel=1e-12)


def test_simulate_open_loop(tg, golden):
    g = golden("newton_iteration")
    assert rel_l2(tg.simulate_open_loop(g["sim_x0"], g["sim_u"]), g["sim_x"]) < 1e-12


# ----------------------------------------------------------------------------- full solves
def test_task2_newton_algorithm_matches_reference_golden(tg, golden, task2_refs):
    """main.task_2's call (main.py:65-71) through the drop-in API reproduces acrobot_optimal_trajectory.npz."""
    xr, ur, _ = task2_refs
    ref = golden("task2_reference_output")
    run = golden("task2_solve")
    x, u, K, sigma, hist = tg.newton_Algorithm(np.array([0, 0, 0, 0]), xr, ur, max_iters=5000, tol=1e-4,
                                               gamma_0=0.1, plot_armijo_iters=7, verbose=False)
    assert x.shape == (501, 4) and u.shape == (500, 2) and len(K) == 500 and K[0].shape == (2, 4)
    assert rel_l2(x, ref["x"]) < TOL_TRAJ
    assert rel_l2(u, ref["u"]) < TOL_TRAJ
    assert len(hist["sigma_norm"]) == 393 and len(hist["cost"]) == 394 and len(hist["x_trajs"]) == 394
    np.testing.assert_allclose(hist["cost"], run["cost_hist"], rtol=1e-9)
    np.testing.assert_allclose(hist["sigma_norm"], run["sigma_norm_hist"], rtol=1e-6)
    assert rel_l2(np.asarray(K), run["K"]) < 1e-8
    assert rel_l2(np.asarray(sigma), run["sigma"]) < 1e-6
    assert rel_l2(np.asarray(hist["sigmas"][0]), run["sigma_first"]) < 1e-10
    for j, i in enumerate(run["x_hist_idx"]):     # iteration 0 is the all-zero open-loop rollout
        np.testing.assert_allclose(hist["x_trajs"][i], run["x_hist"][j], rtol=1e-9, atol=1e-12)


def test_streamed_sigma_is_the_rerun_bit_for_bit(task2_refs):
    """The drop-in newton_Algorithm runs its solver with stream_sigma(): one four-wavefront persistent launch per
    iteration whose sweep stores sigma1, read back by sigma() instead of re-running the sweep.  After every
    iteration that sigma equals the re-run's bit for bit (sign of zero included), and the iterates, costs and
    decisions equal the serial schedule's, on lanes that converge, backtrack and fail the line search."""
    import torch
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr, ur, _ = task2_refs
    x0 = np.zeros((6, 4))
    x0[1, :2] = [1.2, -1.3]
    x0[2, :2] = [2.9, -2.5]
    x0[3, :2] = [0.3, 0.2]
    x0[4, :2] = [-1.4, 1.45]
    x0[5] = np.nan
    eng = AcrobotEngine()
    kw = dict(tol=1e-4, gamma_0=0.1, pipeline=False)
    a = BatchedNewtonSolver(eng, xr, ur, 6, **kw)
    b = BatchedNewtonSolver(eng, xr, ur, 6, **kw)
    a.init(x0)
    a.stream_sigma()
    b.init(x0)
    seen_backtrack = False
    for k in range(120):
        a.iteration()
        b.iteration()
        fast, rerun = a.sigma(), a.sigma(rerun=True)
        assert torch.equal(fast.view(torch.int64), rerun.view(torch.int64)), k
        assert torch.equal(fast.view(torch.int64), b.sigma().view(torch.int64)), k
        for name in ("cost", "status", "n_iter", "n_roll", "gamma", "smax"):
            va, vb = getattr(a, name)[:6], getattr(b, name)[:6]
            assert torch.equal(va.view(torch.int64) if va.is_floating_point() else va,
                               vb.view(torch.int64) if vb.is_floating_point() else vb), (k, name)
        seen_backtrack |= bool((a.n_roll[:6] > a.n_iter[:6]).any())
    assert seen_backtrack
    for ta, tb in zip(a.finalize(), b.finalize()):      # every lane's result iterate, controls, gains, sigma
        assert torch.equal(ta.view(torch.int64), tb.view(torch.int64))


def test_task1_with_live_tau1_channel(tg, golden):
    g = golden("task1_solve")
    x, u, K, sigma, hist = tg.newton_Algorithm(g["x0"], g["x_ref"], g["u_ref_full"], max_iters=5000, tol=1e-4,
                                               gamma_0=0.05, verbose=False)
    assert len(hist["sigma_norm"]) == int(g["n_iter"]) == 173
    assert rel_l2(x, g["x"]) < TOL_TRAJ and rel_l2(u, g["u"]) < TOL_TRAJ
    np.testing.assert_allclose(hist["cost"], g["cost_hist"], rtol=1e-9)


def test_batched_lanes_match_reference_decisions(golden, task2_refs):
    """12 reference lanes incl. backtracking and LS-failure lanes: identical iteration counts, statuses,
    cost / sigma-norm histories, and trajectories within 1e-8."""
    from gymnast_optimalcontrol_amd import _lib
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    L = golden("lanes")
    xr, ur, _ = task2_refs
    B = len(L["names"])
    s = BatchedNewtonSolver(AcrobotEngine(), xr, ur, B, tol=1e-4, gamma_0=0.1, hist_len=900)
    r = s.solve(L["x0"], 5000)
    codes = {1: _lib.CONVERGED, 2: _lib.LS_FAILED}
    n_iter = r.n_iter.cpu().numpy(); status = r.status.cpu().numpy()
    hc = r.hist_cost.cpu().numpy(); hs = r.hist_smax.cpu().numpy()
    for i, name in enumerate(L["names"]):
        n = int(L["n_iter"][i])
        assert n_iter[i] == n, name
        assert status[i] == codes[int(L["status"][i])], name
        np.testing.assert_allclose(hs[:n, i], L["sigma_norm_hist"][i, :n], rtol=1e-6, err_msg=name)
        ncost = n if status[i] == _lib.CONVERGED else n - 1
        np.testing.assert_allclose(hc[:ncost, i], L["cost_hist"][i, 1:ncost + 1], rtol=1e-9, err_msg=name)
        assert rel_l2(r.x[i].cpu().numpy(), L["x"][i]) < TOL_TRAJ, name
        assert rel_l2(r.u[i].cpu().numpy(), L["u"][i]) < TOL_TRAJ, name
        assert rel_l2(r.K[i].cpu().numpy(), L["K"][i]) < 1e-6, name
    assert r.lane_iterations == int(L["n_iter"].sum())


def test_lane_independence_large_batch(golden, task2_refs):
    """Golden lanes embedded in a 65,536-lane batch give the same results; random lanes agree with the
    C oracle on decisions and to 1e-8 on trajectories."""
    from oracle import c_oracle
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    L = golden("lanes")
    xr, ur, _ = task2_refs
    B = 65536
    rng = np.random.default_rng(0)
    x0 = np.zeros((B, 4))
    x0[:, :2] = rng.uniform(-0.5, 0.5, (B, 2))
    idx = np.array([0, 777, 4095, 4096, 30001, 65535, 12, 13, 40000, 40001, 40002, 9])
    x0[idx] = L["x0"]
    r = BatchedNewtonSolver(AcrobotEngine(), xr, ur, B, tol=1e-4, gamma_0=0.1).solve(x0, 5000)
    n_iter = r.n_iter.cpu().numpy()
    for j, i in enumerate(idx):
        assert n_iter[i] == L["n_iter"][j]
        assert rel_l2(r.x[i].cpu().numpy(), L["x"][j]) < TOL_TRAJ
    sample = rng.choice(np.setdiff1d(np.arange(B), idx), 1024, replace=False)   # ~3 s of the C oracle
    o = c_oracle.newton_solve(x0[sample], xr, ur, max_iters=5000, tol=1e-4, gamma_0=0.1)
    np.testing.assert_array_equal(n_iter[sample], o["n_iter"])
    np.testing.assert_array_equal(r.status.cpu().numpy()[sample], o["status"])
    for j, i in enumerate(sample):
        assert rel_l2(r.x[i].cpu().numpy(), o["x"][j]) < TOL_TRAJ
        assert rel_l2(r.u[i].cpu().numpy(), o["u"][j]) < TOL_TRAJ


def test_determinism_bitwise(task2_refs):
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr, ur, _ = task2_refs
    x0 = np.zeros((300, 4)); x0[:, :2] = np.random.default_rng(5).uniform(-1.5, 1.5, (300, 2))
    s = BatchedNewtonSolver(AcrobotEngine(), xr, ur, 300, tol=1e-4, gamma_0=0.1)
    a = s.solve(x0, 60, keep_stats=True)
    b = s.solve(x0, 60, keep_stats=True)
    assert np.array_equal(a.x.cpu().numpy(), b.x.cpu().numpy())
    assert np.array_equal(a.cost.cpu().numpy(), b.cost.cpu().numpy())
    assert np.array_equal(np.asarray(a.stats_log), np.asarray(b.stats_log))


@pytest.mark.parametrize("B", [1, 63, 64, 65, 200])
def test_ragged_batches_and_padding(B, task2_refs):
    """Lane counts that are not multiples of the wavefront: padding lanes never leak into results/stats."""
    from oracle import c_oracle
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr, ur, _ = task2_refs
    x0 = np.zeros((B, 4)); x0[:, :2] = np.random.default_rng(B).uniform(-0.5, 0.5, (B, 2))
    r = BatchedNewtonSolver(AcrobotEngine(), xr, ur, B, tol=1e-4, gamma_0=0.1).solve(x0, 25, keep_stats=True)
    o = c_oracle.newton_solve(x0, xr, ur, max_iters=25, tol=1e-4, gamma_0=0.1)
    np.testing.assert_array_equal(r.n_iter.cpu().numpy(), o["n_iter"])
    np.testing.assert_array_equal(r.status.cpu().numpy(), o["status"])     # all MAX_ITERS after 25
    assert rel_l2(r.x.cpu().numpy(), o["x"]) < 1e-10
    np.testing.assert_allclose(r.cost.cpu().numpy(), o["cost"], rtol=1e-11)
    last = r.stats_log[-1]
    assert last[3] == B and last[0] == B                       # lanes that ran / still active (pre-finalize)
    assert last[1] == pytest.approx(o["cost"].sum(), rel=1e-10)


# Far from convergence (gamma_0 = 1, wide starts) Newton iterates amplify rounding-level differences from one
# iteration to the next.  How much is a property of the problem, measured on runs of the reference itself
# (tests/golden/wide_lanes.npz, make_golden_wide.py, 25 of these lanes): after 120 iterations (every such lane has
# hit its Armijo failure by then) the C restatement's last iterate differs from the reference's by up to 5.5e-6
# (x), 9.4e-6 (u), 1.3e-6 (K) and 2.7e-3 (sigma, the last Newton step, nearly cancelling) per lane -- lane 151
# and 116 -- with every decision identical; after 12 iterations by <= 3e-13.  The bounds below are 10x those
# reference-pinned spreads.  Decisions (iteration counts, statuses, rollout counts) must agree exactly on every
# lane; a sigma taken from the wrong iterate would differ by O(1).
WIDE_TOL = {12: dict(x=1e-11, u=1e-11, K=1e-11, sigma=1e-11, cost=1e-12),
            120: dict(x=6e-5, u=1e-4, K=1.5e-5, sigma=3e-2, cost=2e-6)}


def _decisions_agree(got, ref, what):
    ni, st, nr = got
    bad = np.flatnonzero((ni != ref["n_iter"]) | (st != ref["status"]) | (nr != ref["n_rollouts"]))
    assert bad.size == 0, (f"{what}: decisions differ on lanes {bad.tolist()}: n_iter {ni[bad].tolist()} vs "
                           f"{ref['n_iter'][bad].tolist()}, status {st[bad].tolist()} vs {ref['status'][bad].tolist()}, "
                           f"rollouts {nr[bad].tolist()} vs {ref['n_rollouts'][bad].tolist()}")


def _per_lane(got, ref):
    n = got.shape[0]
    return np.linalg.norm((got - ref).reshape(n, -1), axis=1) / \
        np.maximum(np.linalg.norm(ref.reshape(n, -1), axis=1), 1e-300)


@pytest.mark.parametrize("schedule", ["serial", "pipelined", "persistent"])
@pytest.mark.parametrize("max_iters", [12, 120])
def test_last_iteration_gains_and_sigma_vs_oracle(task2_refs, schedule, max_iters):
    """K and sigma of each lane's last iteration (newton_Algorithm's return values) after backtracking, LS
    failures, a NaN lane and the max_iters cut-off, on 160 wide-start lanes with gamma_0 = 1.  sigma1 is not
    streamed by the solver: gym_newton_sigma re-runs each lane's last sweep from the state buffer that iteration
    started from, and the lanes that backtrack re-run theirs inside the iteration; both must reproduce the
    oracle's values.  Every lane's decisions agree exactly; values within WIDE_TOL per lane."""
    from gymnast_optimalcontrol_amd import _lib
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    from oracle import c_oracle
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden_wide import wide_x0
    xr, ur, _ = task2_refs
    x0 = wide_x0()                                           # lanes 0-19 with initial velocities; lane 9 NaN
    B = x0.shape[0]
    r = BatchedNewtonSolver(AcrobotEngine(), xr, ur, B, tol=1e-4, gamma_0=1.0, pipeline=schedule == "pipelined",
                            persistent=schedule == "persistent").solve(x0, max_iters)
    o = c_oracle.newton_solve(x0, xr, ur, max_iters=max_iters, tol=1e-4, gamma_0=1.0)
    ni, st = r.n_iter.cpu().numpy(), r.status.cpu().numpy()
    _decisions_agree((ni, st, r.n_rollouts.cpu().numpy()), o, f"{schedule}, {max_iters} iterations")
    assert st[9] == _lib.LS_FAILED and np.isnan(r.sigma.cpu().numpy()[9]).any()
    assert (r.n_rollouts.cpu().numpy() > ni).any()                           # some lanes backtracked
    if max_iters == 120:
        assert (st == _lib.LS_FAILED).sum() >= 2
    ok = np.isfinite(o["cost"])
    assert ok.sum() == B - 1
    for name, ref in (("sigma", o["sigma"]), ("K", o["K"]), ("x", o["x"]), ("u", o["u"])):
        err = _per_lane(getattr(r, name).cpu().numpy()[ok], ref[ok])
        tol = WIDE_TOL[max_iters][name]
        assert err.max() < tol, (name, int(np.flatnonzero(ok)[np.argmax(err)]), float(err.max()))


@pytest.mark.parametrize("schedule", ["serial", "pipelined", "persistent"])
@pytest.mark.parametrize("max_iters", [12, 120])
def test_wide_start_lanes_vs_reference(golden, task2_refs, schedule, max_iters):
    """25 lanes like those pinned to the REFERENCE itself (tests/golden/wide_lanes.npz: newton_Algorithm with
    gamma_0 = 1, tol 1e-4, run in the build container): identical iteration counts, statuses and rollout counts
    (backtracking and the Armijo failure of trajectory_generation.py:352-369), and last-iteration K, sigma, x, u
    per lane within 10x the C restatement's own distance from the reference (no looser than WIDE_TOL)."""
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    from oracle import c_oracle
    W = golden("wide_lanes")
    xr, ur, _ = task2_refs
    m = f"m{max_iters}_"
    x0 = W[m + "x0"]
    ref = {"n_iter": W[m + "n_iter"], "status": W[m + "status"], "n_rollouts": W[m + "n_rollouts"]}
    r = BatchedNewtonSolver(AcrobotEngine(), xr, ur, x0.shape[0], tol=1e-4, gamma_0=1.0,
                            pipeline=schedule == "pipelined", persistent=schedule == "persistent").solve(x0, max_iters)
    _decisions_agree((r.n_iter.cpu().numpy(), r.status.cpu().numpy(), r.n_rollouts.cpu().numpy()), ref,
                     f"{schedule} vs reference, {max_iters} iterations")
    o = c_oracle.newton_solve(x0, xr, ur, max_iters=max_iters, tol=1e-4, gamma_0=1.0)
    for name in ("K", "sigma", "x", "u"):
        err = _per_lane(getattr(r, name).cpu().numpy(), W[m + name])
        bound = np.minimum(np.maximum(10 * _per_lane(o[name], W[m + name]), 1e-11), WIDE_TOL[max_iters][name])
        assert (err <= bound).all(), (name, np.flatnonzero(err > bound).tolist(), err.max())
    n, st = W[m + "n_iter"], W[m + "status"]
    # final cost = the last accepted entry of the reference's history['cost']
    J = np.array([W[m + "cost_hist"][i, int(n[i]) - 1 if int(st[i]) == 2 else int(n[i])] for i in range(len(n))])
    err = np.abs(r.cost.cpu().numpy() - J) / np.abs(J)
    bound = np.minimum(np.maximum(10 * np.abs(o["cost"] - J) / np.abs(J), 1e-12), WIDE_TOL[max_iters]["cost"])
    assert (err <= bound).all(), ("cost", np.flatnonzero(err > bound).tolist(), err.max())


def test_single_trial_line_search_and_nan_lane(task2_refs):
    """max_ls = 1 (no retry path) and a NaN initial state (NaN costs compare false -> LS failure)."""
    from gymnast_optimalcontrol_amd import _lib
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    from oracle import c_oracle
    xr, ur, _ = task2_refs
    x0 = np.zeros((4, 4)); x0[1, :2] = [1.2, -1.0]; x0[2] = np.nan; x0[3, :2] = [-1.4, 1.4]
    r = BatchedNewtonSolver(AcrobotEngine(), xr, ur, 4, tol=1e-4, gamma_0=1.0, max_ls=1).solve(x0, 200)
    o = c_oracle.newton_solve(x0, xr, ur, max_iters=200, tol=1e-4, gamma_0=1.0, max_ls=1)
    np.testing.assert_array_equal(r.n_iter.cpu().numpy(), o["n_iter"])
    np.testing.assert_array_equal(r.status.cpu().numpy(), o["status"])
    assert int(r.status[2]) == _lib.LS_FAILED and int(r.n_iter[2]) == 1
    ok = np.isfinite(o["cost"])
    assert rel_l2(r.x.cpu().numpy()[ok], o["x"][ok]) < 1e-9


def test_u_ref_trim_and_errors(tg, task2_refs):
    xr, ur, _ = task2_refs
    ur_full = np.vstack([ur, ur[-1:]])               # N rows -> trimmed (:301-303)
    x1, u1, *_ = tg.newton_Algorithm(np.zeros(4), xr, ur_full, max_iters=3, tol=1e-4, gamma_0=0.1, verbose=False)
    x2, u2, *_ = tg.newton_Algorithm(np.zeros(4), xr, ur, max_iters=3, tol=1e-4, gamma_0=0.1, verbose=False)
    assert np.array_equal(x1, x2) and np.array_equal(u1, u2)
    with pytest.raises(ValueError, match="Incompatible dimensions"):
        tg.newton_Algorithm(np.zeros(4), xr, ur[:-3], max_iters=3)


@pytest.mark.parametrize("persistent", [False, True])
def test_full_size_properties(task2_refs, persistent):
    """BASELINE cfg 3 exactly as bench.py runs it (262,144 lanes, bench.make_x0): EVERY lane's iteration count,
    status and rollout count equal to the C oracle's and its final cost within 1e-11 (tests/golden/
    headline_oracle.npz, the C oracle over the whole batch, make_headline_oracle.py); the golden lane 0 within 1e-8
    of the reference's trajectory; the statistics consistent; 1,024 lanes spread over the batch within 1e-8 of the
    oracle's trajectories (run live: trajectories are not in the fixture).  No lane backtracks on this workload, so
    the pipelined solver never allocates its candidate scratch."""
    from bench import make_x0
    from conftest import load_golden
    from gymnast_optimalcontrol_amd import _lib
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr, ur, _ = task2_refs
    B = 262144
    x0 = make_x0(B)
    s = BatchedNewtonSolver(AcrobotEngine(), xr, ur, B, tol=1e-4, gamma_0=0.1, persistent=persistent)
    r = s.solve(x0, 5000, keep_stats=True)
    assert s._cand_scratch is None
    ref = load_golden("task2_reference_output")
    assert rel_l2(r.x[0].cpu().numpy(), ref["x"]) < TOL_TRAJ
    st = r.status.cpu().numpy(); n = r.n_iter.cpu().numpy(); nr = r.n_rollouts.cpu().numpy()
    cost = r.cost.cpu().numpy()
    assert (st == _lib.CONVERGED).all()
    assert 370 <= n.min() and n.max() <= 420
    assert r.lane_iterations == int(n.sum())
    if not persistent:   # one statistics row per iteration: "lanes that ran" sums to the lane-iterations
        assert r.lane_iterations == int(sum(s[3] for s in r.stats_log))
    else:
        assert r.stats_log[-1][0] == 0 and r.stats_log[-1][5] == B
    o = load_golden("headline_oracle")
    assert float(o["spread"]) == 0.5 and len(o["n_iter"]) == B
    np.testing.assert_array_equal(n, o["n_iter"])
    np.testing.assert_array_equal(st, o["status"])
    np.testing.assert_array_equal(nr, o["n_rollouts"])
    assert (o["k_tie"] < 0).all()          # no Armijo test of the headline workload is near a tie
    rel = np.abs(cost - o["cost"]) / np.abs(o["cost"])
    assert rel.max() < 1e-11, rel.max()
    from oracle import c_oracle
    pick = np.linspace(0, B - 1, 1024).astype(np.int64)
    oc = c_oracle.newton_solve(x0[pick], xr, ur, max_iters=5000, tol=1e-4, gamma_0=0.1)
    np.testing.assert_array_equal(n[pick], oc["n_iter"])
    xs, us = r.x[pick].cpu().numpy(), r.u[pick].cpu().numpy()
    ex = np.linalg.norm((xs - oc["x"]).reshape(1024, -1), axis=1) / np.linalg.norm(oc["x"].reshape(1024, -1), axis=1)
    eu = np.linalg.norm((us - oc["u"]).reshape(1024, -1), axis=1) / np.linalg.norm(oc["u"].reshape(1024, -1), axis=1)
    assert ex.max() < TOL_TRAJ and eu.max() < TOL_TRAJ, (ex.max(), eu.max())


@pytest.mark.parametrize("max_iters", [25, 5000])
def test_pipelined_schedule_matches_serial(task2_refs, max_iters):
    """The two-half pipelined schedule (gym_newton_phase) gives bitwise the serial schedule's lanes,
    including backtracking / LS-failure lanes and the max_iters cut-off (last-iteration K and sigma)."""
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr, ur, _ = task2_refs
    B = 1000
    x0 = np.zeros((B, 4)); x0[:, :2] = np.random.default_rng(21).uniform(-1.5, 1.5, (B, 2))
    x0[7] = np.nan
    eng = AcrobotEngine()
    rs = BatchedNewtonSolver(eng, xr, ur, B, tol=1e-4, gamma_0=0.1, pipeline=False).solve(x0, max_iters, keep_stats=True)
    rp = BatchedNewtonSolver(eng, xr, ur, B, tol=1e-4, gamma_0=0.1, pipeline=True).solve(x0, max_iters, keep_stats=True)
    for name in ("x", "u", "K", "sigma", "cost", "n_iter", "status", "n_rollouts", "gamma"):
        a, b = getattr(rs, name).cpu().numpy(), getattr(rp, name).cpu().numpy()
        assert np.array_equal(a, b, equal_nan=True), name
    assert rs.iterations == rp.iterations
    ls, lp = np.asarray(rs.stats_log), np.asarray(rp.stats_log)
    np.testing.assert_array_equal(ls[:, [0, 3, 4, 5, 6, 7]], lp[:, [0, 3, 4, 5, 6, 7]])   # counts: exact
    np.testing.assert_allclose(ls[:, [1, 2]], lp[:, [1, 2]], rtol=1e-12)                  # sums: order differs
    if max_iters == 5000:
        assert (rs.status.cpu().numpy() == 2).sum() >= 2        # the batch exercises LS failures
        assert ls[:, 4].sum() > 0                               # ... and Armijo retries


@pytest.mark.parametrize("max_iters,chunk,u0z", [(25, 0, True), (5000, 0, True), (5000, 7, False), (5000, 0, False)])
@pytest.mark.parametrize("split", [True, False])
def test_persistent_schedule_matches_serial(task2_refs, max_iters, chunk, u0z, split):
    """The persistent schedule (gym_newton_run: each lane's iterations back to back in one launch per chunk, its
    Armijo trials 2..max_ls sequential) gives bitwise the serial schedule's lanes -- trajectories, last-iteration
    K and sigma, costs, decisions, rollout counts, per-lane histories -- incl. backtracking / LS-failure / NaN
    lanes, the max_iters cut-off and chunked launches -- on the two-wavefront kernel (k_nt_run2, default) and the
    single-wavefront one (GYM_FLAG_RUN_SINGLE)."""
    from gymnast_optimalcontrol_amd import _lib
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr, ur, _ = task2_refs
    B = 1000
    x0 = np.zeros((B, 4)); x0[:, :2] = np.random.default_rng(21).uniform(-1.5, 1.5, (B, 2))
    x0[7] = np.nan
    eng = AcrobotEngine()
    kw = dict(tol=1e-4, gamma_0=0.1, u0_zero=None if u0z else False, hist_len=64)
    rs = BatchedNewtonSolver(eng, xr, ur, B, pipeline=False, **kw).solve(x0, max_iters, keep_stats=True)
    rr = BatchedNewtonSolver(eng, xr, ur, B, persistent=True, chunk=chunk, split_waves=split,
                             **kw).solve(x0, max_iters, keep_stats=True)
    for name in ("x", "u", "K", "sigma", "cost", "n_iter", "status", "n_rollouts", "gamma", "hist_cost", "hist_smax"):
        a, b = getattr(rs, name).cpu().numpy(), getattr(rr, name).cpu().numpy()
        assert np.array_equal(a, b, equal_nan=True), name
    assert rs.iterations == rr.iterations
    last_s, last_r = rs.stats_log[-1], rr.stats_log[-1]
    np.testing.assert_array_equal(last_s[[0, 5, 6, 7]], last_r[[0, 5, 6, 7]])   # active, converged, failed, rollouts
    np.testing.assert_allclose(last_s[1], last_r[1], rtol=1e-12)                 # sum J (summation order differs)
    st = rr.status.cpu().numpy()
    if max_iters == 5000:
        assert (st == _lib.LS_FAILED).sum() >= 2 and st[7] == _lib.LS_FAILED
        assert (rr.n_rollouts.cpu().numpy() > rr.n_iter.cpu().numpy()).sum() > 0   # Armijo retries happened
    else:
        assert (st == _lib.MAX_ITERS).any()


@pytest.mark.parametrize("N", [2, 3, 4, 6, 37, 203])
def test_every_schedule_on_short_and_ragged_horizons(task2_refs, N):
    """Horizons from one stage (N = 2) up, odd ones, and ones shorter than the persistent kernel's chunk (2 stages)
    and prefetch distance (4 stages) or the ILP sweep's unroll (6): the serial, pipelined and persistent (four- and
    single-wavefront) solves are bitwise equal, lane by lane (incl. a NaN lane); the serial one has the C oracle's
    decisions and its trajectories within 1e-8; a one-lane batch is bitwise its lane of the 130-lane batch."""
    from gymnast_optimalcontrol_amd import _lib
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    from oracle import c_oracle
    xr, ur, _ = task2_refs
    xr, ur = xr[:N], ur[:N - 1]
    B, max_iters = 130, 300
    x0 = np.zeros((B, 4)); x0[:, :2] = np.random.default_rng(60 + N).uniform(-1.5, 1.5, (B, 2))
    x0[3] = np.nan
    eng = AcrobotEngine()
    kw = dict(tol=1e-4, gamma_0=0.1, hist_len=16)
    names = ("x", "u", "K", "sigma", "cost", "n_iter", "status", "n_rollouts", "gamma", "hist_cost", "hist_smax")
    rs = BatchedNewtonSolver(eng, xr, ur, B, pipeline=False, persistent=False, **kw).solve(x0, max_iters)
    assert rs.schedule == "serial"
    for sched in (dict(pipeline=True), dict(persistent=True), dict(persistent=True, split_waves=False)):
        r = BatchedNewtonSolver(eng, xr, ur, B, **sched, **kw).solve(x0, max_iters)
        for name in names:
            assert np.array_equal(getattr(rs, name).cpu().numpy(), getattr(r, name).cpu().numpy(),
                                  equal_nan=True), (sched, name)
    for sched in (dict(pipeline=False, persistent=False), dict(pipeline=True), dict(persistent=True)):
        r1 = BatchedNewtonSolver(eng, xr, ur, 1, **sched, **kw).solve(x0[5:6], max_iters)
        for name in names:
            a = getattr(rs, name).cpu().numpy()
            a = a[:, 5:6] if name.startswith("hist") else a[5:6]
            assert np.array_equal(a, getattr(r1, name).cpu().numpy(), equal_nan=True), (sched, name)
    st = rs.status.cpu().numpy()
    assert st[3] == _lib.LS_FAILED
    ok = np.arange(B) != 3
    o = c_oracle.newton_solve(x0[ok], xr, ur, max_iters=max_iters, tol=1e-4, gamma_0=0.1)
    np.testing.assert_array_equal(rs.n_iter.cpu().numpy()[ok], o["n_iter"])
    np.testing.assert_array_equal(st[ok], o["status"])
    np.testing.assert_array_equal(rs.n_rollouts.cpu().numpy()[ok], o["n_rollouts"])
    for name in ("x", "u"):
        a, e = getattr(rs, name).cpu().numpy()[ok].reshape(B - 1, -1), o[name].reshape(B - 1, -1)
        assert (np.linalg.norm(a - e, axis=1) / np.linalg.norm(e, axis=1)).max() < TOL_TRAJ, name


@pytest.mark.parametrize("pipeline", [False, True])
def test_lane_reordering_is_invisible(task2_refs, pipeline):
    """solve() runs the lanes in the Morton order of their initial states and writes the results back in the
    caller's order: bitwise the results of the unreordered solve, lane by lane (incl. NaN / LS-failure lanes)."""
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr, ur, _ = task2_refs
    B = 700
    x0 = np.zeros((B, 4)); x0[:, :2] = np.random.default_rng(51).uniform(-1.5, 1.5, (B, 2))
    x0[11] = np.nan
    eng = AcrobotEngine()
    kw = dict(tol=1e-4, gamma_0=0.1, pipeline=pipeline, hist_len=32)
    ra = BatchedNewtonSolver(eng, xr, ur, B, reorder=True, **kw).solve(x0, 5000)
    rb = BatchedNewtonSolver(eng, xr, ur, B, reorder=False, **kw).solve(x0, 5000)
    for name in ("x", "u", "K", "sigma", "cost", "n_iter", "status", "n_rollouts", "gamma", "hist_cost", "hist_smax"):
        a, b = getattr(ra, name).cpu().numpy(), getattr(rb, name).cpu().numpy()
        assert np.array_equal(a, b, equal_nan=True), name


def test_persistent_schedule_refuses_checkpointing(task2_refs):
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr, ur, _ = task2_refs
    with pytest.raises(ValueError):
        BatchedNewtonSolver(AcrobotEngine(), xr, ur, 8, persistent=True, checkpoint=True)


@pytest.mark.parametrize("pipeline", [False, True])
def test_u0_zero_stream_skipping_is_bitwise_identical(task2_refs, pipeline):
    """GYM_FLAG_U0_ZERO (u_ref[:,0] == 0: tau1 planes neither read nor written) gives bitwise the general
    path's results, incl. backtracking / LS-failure / NaN lanes; it is refused when u_ref[:,0] != 0."""
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr, ur, _ = task2_refs
    assert (ur[:, 0] == 0).all()
    B = 700
    x0 = np.zeros((B, 4)); x0[:, :2] = np.random.default_rng(33).uniform(-1.5, 1.5, (B, 2))
    x0[3] = np.nan
    eng = AcrobotEngine()
    sz = BatchedNewtonSolver(eng, xr, ur, B, tol=1e-4, gamma_0=0.1, pipeline=pipeline)
    sg = BatchedNewtonSolver(eng, xr, ur, B, tol=1e-4, gamma_0=0.1, pipeline=pipeline, u0_zero=False)
    assert sz.u0_zero and not sg.u0_zero
    rz, rg = sz.solve(x0, 5000, keep_stats=True), sg.solve(x0, 5000, keep_stats=True)
    for name in ("x", "u", "K", "sigma", "cost", "n_iter", "status", "n_rollouts", "gamma"):
        a, b = getattr(rz, name).cpu().numpy(), getattr(rg, name).cpu().numpy()
        assert np.array_equal(a, b, equal_nan=True), name
    assert (rz.u.cpu().numpy()[:, :, 0] == 0).all()
    assert np.array_equal(np.asarray(rz.stats_log), np.asarray(rg.stats_log), equal_nan=True)
    ur1 = ur.copy(); ur1[5, 0] = 0.25
    assert not BatchedNewtonSolver(eng, xr, ur1, 4).u0_zero
    with pytest.raises(ValueError):
        BatchedNewtonSolver(eng, xr, ur1, 4, u0_zero=True)


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline,u0z,N", [(False, True, 501), (True, True, 501), (False, False, 501),
                                            (True, False, 203), (False, True, 6)])
def test_state_checkpointing_is_bitwise_identical(task2_refs, pipeline, u0z, N):
    """GYM_FLAG_X_CKPT (trials store every 4th knot, the sweep re-integrates the rest) gives bitwise the
    full-store path's results -- trajectories, gains, sigma, costs, decisions, statistics -- incl. ragged
    horizons (T % 4 != 0, T < 4) and backtracking / LS-failure / NaN lanes; states() rebuilds a buffer
    mid-solve to the full-store buffer's bits."""
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr, ur, _ = task2_refs
    xr, ur = xr[:N], ur[:N - 1]
    B = 600
    x0 = np.zeros((B, 4)); x0[:, :2] = np.random.default_rng(44).uniform(-1.5, 1.5, (B, 2))
    x0[5] = np.nan
    eng = AcrobotEngine()
    kw = dict(tol=1e-4, gamma_0=0.1, pipeline=pipeline, u0_zero=None if u0z else False)
    sc = BatchedNewtonSolver(eng, xr, ur, B, checkpoint=True, **kw)
    sf = BatchedNewtonSolver(eng, xr, ur, B, checkpoint=False, **kw)
    # mid-solve: 7 iterations, then the rebuilt current buffer equals the full-store one
    for s in (sc, sf):
        s.max_iters = 5000
        s.init(x0)
        for _ in range(7):
            s.iteration()
    buf = (7 & 1)
    assert np.array_equal(eng.unpack(sc.states(buf), B).cpu().numpy(), eng.unpack(sf.states(buf), B).cpu().numpy(),
                          equal_nan=True)
    rc, rf = sc.solve(x0, 5000, keep_stats=True), sf.solve(x0, 5000, keep_stats=True)
    for name in ("x", "u", "K", "sigma", "cost", "n_iter", "status", "n_rollouts", "gamma"):
        a, b = getattr(rc, name).cpu().numpy(), getattr(rf, name).cpu().numpy()
        assert np.array_equal(a, b, equal_nan=True), name
    assert np.array_equal(np.asarray(rc.stats_log), np.asarray(rf.stats_log), equal_nan=True)


@pytest.mark.parametrize("C,W", [(1, 1), (2, 2), (2, 1), (3, 1), (4, 2), (6, 2), (8, 2), (8, 1), (12, 2), (13, 1)])
def test_lane_transposes_round_trip(eng, C, W):
    """gym_pack_lanes -> gym_unpack_lanes is the identity, bitwise, on a ragged batch over several LDS tiles of
    knots: the compile-time component counts of the tiled unpack (2, 4, 8) and its run-time form, pairs and planes,
    and the per-lane src0 / src1 select."""
    import torch
    B, L = 200, 501
    Bp = (B + 63) // 64 * 64
    g = torch.Generator().manual_seed(10 * C + W)
    a = torch.randn(B, L, C, generator=g, dtype=torch.float64)
    b = torch.randn(B, L, C, generator=g, dtype=torch.float64)
    sa, sb = eng.pack(a.to(eng.device), Bp, W), eng.pack(b.to(eng.device), Bp, W)
    if W == 1:
        assert not sa[:, :, B:, :].any()          # padding lanes are zero-filled
    assert torch.equal(eng.unpack(sa, B).cpu(), a)
    sel = (torch.arange(B) % 3 == 1).to(torch.int32)
    got = eng.unpack(sa, B, sb, sel.to(eng.device)).cpu()
    assert torch.equal(got, torch.where(sel.bool()[:, None, None], b, a))


def test_per_lane_references(golden, task2_refs):
    """Per-lane references (SURVEY 8(b)'s batched form: x_ref (B,N,4), u_ref (B,T,2); GYM_FLAG_REF_LANE, every
    schedule): three references dealt round-robin over 150 lanes -- task 2's, task 2's with 0.8 u_ref, and task 1's
    (a live tau1 channel) -- in Morton order.  Every lane is bit for bit the lane of the shared-reference solve of
    its group, and the serial, pipelined and single-wavefront persistent solves bit for bit the default
    (persistent, four wavefronts per 64 lanes) one; lane 0 (task 2's reference, x0 = 0) is the reference's task-2
    trajectory."""
    from gymnast_optimalcontrol_amd import _lib
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr2, ur2, _ = task2_refs
    g1 = golden("task1_solve")
    refs = [(xr2, ur2), (xr2, 0.8 * ur2), (g1["x_ref"], g1["u_ref_full"][:-1])]
    B = 150
    x0 = np.zeros((B, 4)); x0[:, :2] = np.random.default_rng(31).uniform(-0.5, 0.5, (B, 2))
    x0[0] = 0.0
    x0[2] = g1["x0"]
    which = np.arange(B) % 3
    XR = np.stack([refs[w][0] for w in which]); UR = np.stack([refs[w][1] for w in which])
    eng = AcrobotEngine()
    kw = dict(tol=1e-4, gamma_0=0.1, hist_len=450)
    s = BatchedNewtonSolver(eng, XR, UR, B, **kw)
    assert s.schedule == "persistent" and s.ref_lane and not s.u0_zero
    r = s.solve(x0, 450)
    st = r.status.cpu().numpy()
    assert (st[which == 0] == _lib.CONVERGED).all(), np.bincount(st[which == 0])
    for w, (xr, ur) in enumerate(refs):
        lanes = np.flatnonzero(which == w)
        rg = BatchedNewtonSolver(eng, xr, ur, lanes.size, **kw).solve(x0[lanes], 450)
        for name in ("x", "u", "K", "sigma", "cost", "n_iter", "status", "n_rollouts", "hist_cost", "hist_smax"):
            a = getattr(r, name).cpu().numpy()
            a = a[:, lanes] if name.startswith("hist") else a[lanes]
            assert np.array_equal(a, getattr(rg, name).cpu().numpy(), equal_nan=True), (w, name)
    g = golden("task2_reference_output")
    assert rel_l2(r.x[0].cpu().numpy(), g["x"]) < TOL_TRAJ and int(r.n_iter[0].item()) == 393
    for sched in (dict(pipeline=False, persistent=False), dict(pipeline=True), dict(split_waves=False)):
        rp = BatchedNewtonSolver(eng, XR, UR, B, **sched, **kw).solve(x0, 450)
        for name in ("x", "u", "K", "sigma", "cost", "n_iter", "status", "n_rollouts", "hist_cost", "hist_smax"):
            assert np.array_equal(getattr(r, name).cpu().numpy(), getattr(rp, name).cpu().numpy(),
                                  equal_nan=True), (sched, name)
    with pytest.raises(ValueError):
        BatchedNewtonSolver(eng, XR, UR, B, checkpoint=True, **kw)
    with pytest.raises(ValueError):
        BatchedNewtonSolver(eng, XR[:10], UR[:10], B, **kw)


def test_placement_selection_is_invisible(task2_refs):
    """Placement selection (round 6: the first solve runs blocks of PLACEMENT_BLOCK iterations on each of up to
    PLACEMENT_TRIALS stream-buffer sets, the live state copied from set to set, and keeps the fastest) changes where the
    streams live, not what they compute: the solve that selects is bit for bit the solve of a solver that kept its
    first allocation, on a batch with backtracking, LS-failure and NaN lanes and per-lane histories.  The chosen set is
    pooled for the process (PlacementPool): a second solver of the same shape takes it at construction (no probe, no
    allocation of streams: < 50 ms) and solves to the same bits."""
    import gc
    import time
    import torch
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver, PlacementPool
    xr, ur, _ = task2_refs
    B, H = 2000, 120
    x0 = np.zeros((B, 4)); x0[:, :2] = np.random.default_rng(5).uniform(-1.5, 1.5, (B, 2))
    x0[11] = np.nan
    eng = AcrobotEngine()
    kw = dict(tol=1e-4, gamma_0=1.0, pipeline=True, hist_len=H)     # gamma_0 = 1: wide starts backtrack early
    trials = BatchedNewtonSolver.PLACEMENT_TRIALS
    assert trials * 2 * BatchedNewtonSolver.PLACEMENT_BLOCK < H
    PlacementPool.clear()
    a = BatchedNewtonSolver(eng, xr, ur, B, placement_trials=1, **kw)
    s = BatchedNewtonSolver(eng, xr, ur, B, placement_trials=trials, **kw)
    assert a.placement is None and s.placement["state"] == "pending" and s.placement["trials"] == trials
    ra, rs = a.solve(x0, H), s.solve(x0, H)
    assert s.placement["state"] == "chosen" and 0 <= s.placement["chosen"] < trials, s.placement
    assert s.placement["probe_iterations"] == 2 * trials * BatchedNewtonSolver.PLACEMENT_BLOCK
    assert s.x[0].data_ptr() == s.batch.x[0] and s.K1.data_ptr() == s.batch.K1 and s.cs.data_ptr() == s.batch.cs
    names = ("x", "u", "K", "sigma", "cost", "n_iter", "status", "n_rollouts", "gamma", "hist_cost", "hist_smax")
    for name in names:
        assert np.array_equal(getattr(ra, name).cpu().numpy(), getattr(rs, name).cpu().numpy(), equal_nan=True), name
    assert (ra.n_rollouts > ra.n_iter).sum().item() > 10 and (ra.status == 2).sum().item() > 0
    chosen_ptr = s.K1.data_ptr()
    del s, rs
    gc.collect()
    assert PlacementPool.held_bytes() > 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s2 = BatchedNewtonSolver(eng, xr, ur, B, placement_trials=trials, **kw)
    torch.cuda.synchronize()
    setup = time.perf_counter() - t0
    assert s2.placement.get("reused") and s2.K1.data_ptr() == chosen_ptr and setup < 0.05, (s2.placement, setup)
    r2 = s2.solve(x0, H)
    for name in names:
        assert np.array_equal(getattr(ra, name).cpu().numpy(), getattr(r2, name).cpu().numpy(), equal_nan=True), name
    del s2
    gc.collect()
    PlacementPool.clear()
    assert PlacementPool.held_bytes() == 0
