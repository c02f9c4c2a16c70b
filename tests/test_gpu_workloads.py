"""BASELINE configurations at their own sizes, parameter sets 2 / 3, selected-lane trajectory capture and the
sharded (multi-rank) solve on the HIP path -- all through the C-ABI, checked against the oracles and the
reference-produced fixtures.

Tolerances: decisions (iteration counts, statuses, rollout counts) exact; converged trajectories 1e-8 rel-L2
(north star); tracking 1e-9 (test_tracking.py); sharded vs unsharded bit for bit (lanes are independent and
every schedule is bitwise-equal per lane).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, load_golden, rel_l2

pytestmark = pytest.mark.gpu

TOL_TRAJ = 1e-8


def _lane_rel(a, b):
    a = a.reshape(a.shape[0], -1); b = b.reshape(b.shape[0], -1)
    return np.linalg.norm(a - b, axis=1) / np.maximum(np.linalg.norm(b, axis=1), 1e-300)


# ----------------------------------------------------------------------------- BASELINE cfg 2
def test_cfg2_full_size_matches_c_oracle():
    """BASELINE cfg 2 exactly as bench.py runs it: 4,096 randomised-theta0 lanes (lane 0 = the golden lane),
    task-2 settings, the default schedule, solved to convergence.  Every lane: identical iteration count,
    status and rollout count; trajectory and controls within 1e-8; lane 0 against the reference's npz."""
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    from oracle import c_oracle
    x_ref, u_ref = load_refs()
    B = 4096
    x0 = make_x0(B)
    s = BatchedNewtonSolver(AcrobotEngine(), x_ref, u_ref, B, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20)
    assert s.schedule == "persistent"                      # the schedule bench.py's cfg 2 line uses
    r = s.solve(x0, 5000)
    o = c_oracle.newton_solve(x0, x_ref, u_ref, max_iters=5000, tol=1e-4, gamma_0=0.1)
    np.testing.assert_array_equal(r.n_iter.cpu().numpy(), o["n_iter"])
    np.testing.assert_array_equal(r.status.cpu().numpy(), o["status"])
    np.testing.assert_array_equal(r.n_rollouts.cpu().numpy(), o["n_rollouts"])
    assert (o["status"] == 1).all()
    ex, eu = _lane_rel(r.x.cpu().numpy(), o["x"]), _lane_rel(r.u.cpu().numpy(), o["u"])
    assert ex.max() < TOL_TRAJ and eu.max() < TOL_TRAJ, (ex.max(), eu.max())
    np.testing.assert_allclose(r.cost.cpu().numpy(), o["cost"], rtol=1e-9)
    g = load_golden("task2_reference_output")
    assert rel_l2(r.x[0].cpu().numpy(), g["x"]) < TOL_TRAJ and rel_l2(r.u[0].cpu().numpy(), g["u"]) < TOL_TRAJ


# ----------------------------------------------------------------------------- BASELINE cfg 4 (one GPU)
def test_cfg4_rank_share_and_pooled_resolve():
    """One rank's share of BASELINE cfg 4 at N = 8 (bench.py's cfg4_rank_share leg): lanes [0, 131072) of the cfg 4
    batch, the schedule every rank of that job picks (distributed.schedule_lanes: pipelined, exactly its 512 lanes
    per CU), with placement selection inside the first solve.  Every lane takes the C oracle's decisions and final
    cost (the fixture's first 131,072 lanes: make_x0 draws the cfg 4 rows as the cfg 3 ones).  Then the batched
    newton_Algorithm's one-shot pattern: the solver goes, a new solver of the same shape takes the pooled stream set
    (no selection) and solves to the same bits."""
    import gc
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd import distributed as gd
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver, PlacementPool
    x_ref, u_ref = load_refs()
    lo, hi = gd.shard_range(1 << 20, 0, 8)
    x0 = make_x0(1 << 20)[lo:hi]
    eng = AcrobotEngine()
    kw = dict(tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20, schedule_lanes=gd.schedule_lanes(1 << 20, 8))
    PlacementPool.clear()
    s = BatchedNewtonSolver(eng, x_ref, u_ref, hi - lo, **kw)
    assert s.schedule == "pipelined" and s.placement["state"] == "pending"
    r = s.solve(x0, 5000, sync_every=4)
    assert s.placement["state"] == "chosen", s.placement
    fx = load_golden("headline_oracle")
    ni, st, nr = (t.cpu().numpy() for t in (r.n_iter, r.status, r.n_rollouts))
    np.testing.assert_array_equal(ni, fx["n_iter"][lo:hi])
    np.testing.assert_array_equal(st, fx["status"][lo:hi])
    np.testing.assert_array_equal(nr, fx["n_rollouts"][lo:hi])
    rel = np.abs(r.cost.cpu().numpy() - fx["cost"][lo:hi]) / np.abs(fx["cost"][lo:hi])
    assert rel.max() < 1e-11, rel.max()
    keep = {k: getattr(r, k)[::97].cpu().numpy() for k in ("x", "u", "K", "sigma", "cost")}
    del r, s
    gc.collect()
    s2 = BatchedNewtonSolver(eng, x_ref, u_ref, hi - lo, **kw)
    assert s2.placement.get("reused"), s2.placement
    r2 = s2.solve(x0, 5000, sync_every=4)
    for k, v in keep.items():
        assert np.array_equal(getattr(r2, k)[::97].cpu().numpy(), v), k
    del r2, s2
    gc.collect()
    PlacementPool.clear()


def test_two_wavefront_phase_kernel_is_bitwise_the_four_wavefront_one():
    """gym_newton_phase picks its two-wavefront build (compiled for two wavefronts per SIMD, both stage loops
    prefetching two stages ahead) for batches of more than 7/8 and at most two wavefronts per SIMD, e.g. the
    131,072 lanes of one rank's cfg 4 share, and its four-wavefront build for the headline 262,144.  Same arithmetic
    in the same order: lanes [0, 131072) of a 262,144-lane solve and 131,072-lane solves on each instantiation of the
    two-wavefront build (shared references with the tau1 planes skipped, the general kernels that stream them, and
    per-lane references) agree bit for bit in every output: iteration counts, statuses and rollouts on every lane;
    x, u, K, sigma and cost on every 97th lane.  Twice: the headline batch to convergence, and the stress start
    (th ~ U(+-1.5): backtracking, the retry kernels after the phases) for 150 iterations."""
    import gc
    import torch
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    x_ref, u_ref = load_refs()
    eng = AcrobotEngine()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    kw = dict(tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20, placement_trials=1)
    H = 131072

    def run(B, x0, iters, u0_zero=None, per_lane=False):
        xr, ur = x_ref, u_ref
        if per_lane:
            xr = np.broadcast_to(x_ref, (B,) + x_ref.shape).copy()
            ur = np.broadcast_to(u_ref, (B,) + u_ref.shape).copy()
        s = BatchedNewtonSolver(eng, xr, ur, B, u0_zero=u0_zero, **kw)
        assert s.schedule == "pipelined"
        waves, simds = B // 64, 4 * cus
        want = "two-wavefront" if 8 * waves > 14 * simds and waves <= 2 * simds else "four-wavefront"
        assert s.phase_kind() == want, (B, cus, s.phase_kind())
        if cus == 256:                           # MI355X: the rank share on the two-wavefront build, the headline not
            assert want == ("two-wavefront" if B == H else "four-wavefront")
        r = s.solve(x0[:B], iters, sync_every=4)
        out = {k: getattr(r, k)[:H].cpu().numpy() for k in ("n_iter", "status", "n_rollouts")}
        out.update({k: getattr(r, k)[:H:97].cpu().numpy() for k in ("x", "u", "K", "sigma", "cost")})
        del r, s
        gc.collect()
        return out

    for spread, iters in ((0.5, 5000), (1.5, 150)):
        x0 = make_x0(2 * H, spread=spread)
        ref = run(2 * H, x0, iters)
        if spread == 1.5:
            assert (ref["n_rollouts"] > ref["n_iter"]).any()      # lanes backtracked
        for case in (dict(), dict(u0_zero=False), dict(per_lane=True)):
            got = run(H, x0, iters, **case)
            for k, v in ref.items():
                assert np.array_equal(got[k], v, equal_nan=True), (spread, case, k)


@pytest.mark.parametrize("N", [202, 203, 4])
def test_two_wavefront_phase_kernel_every_stage_remainder(N):
    """The two-wavefront build's stage loops run three stages per trip and then the remaining T mod 3 (the headline's
    T = 500 leaves 2): horizons T = 201, 202 and 3 (the reference trajectory cut to N knots) leave 0, 1 and 0 with a
    single trip, and give bit for bit the four-wavefront build's results (lanes [0, 131072) of a 262,144-lane solve
    against the 131,072-lane solve, 30 iterations; every lane's counts, every 97th lane's trajectories)."""
    import gc
    import torch
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    x_ref, u_ref = load_refs()
    x_ref, u_ref = x_ref[:N].copy(), u_ref[:N - 1].copy()
    eng = AcrobotEngine()
    H = 131072
    x0 = make_x0(2 * H)
    out = []
    for B in (2 * H, H):
        s = BatchedNewtonSolver(eng, x_ref, u_ref, B, tol=1e-4, gamma_0=0.1, placement_trials=1, pipeline=True)
        if torch.cuda.get_device_properties(0).multi_processor_count == 256:     # MI355X
            assert s.phase_kind() == ("two-wavefront" if B == H else "four-wavefront")
        r = s.solve(x0[:B], 30, sync_every=4)
        o = {k: getattr(r, k)[:H].cpu().numpy() for k in ("n_iter", "status", "n_rollouts")}
        o.update({k: getattr(r, k)[:H:97].cpu().numpy() for k in ("x", "u", "K", "sigma", "cost")})
        out.append(o)
        del r, s
        gc.collect()
    for k, v in out[0].items():
        assert np.array_equal(out[1][k], v, equal_nan=True), (N, k)


def test_cfg4_global_batch_on_one_gpu():
    """BASELINE cfg 4's whole batch, 1,048,576 lanes (bench.py's strong-scaling workload at N = 1; the pipelined
    schedule), solved to convergence on one GPU, checked through size-independent properties: every lane
    converges; lanes 0..4095 (make_x0 draws the same rows for any batch size) are bit for bit the cfg 2 solve of
    those 4,096 lanes (persistent schedule: per-lane results do not depend on the batch, its size or the
    schedule); the first 262,144 lanes (bench.make_x0 draws them as the cfg 3 batch) take exactly the C oracle's
    decisions and its final costs within 1e-11, lane by lane (tests/golden/headline_oracle.npz); 1,024 lanes spread
    over the whole batch match the live C oracle's decisions and trajectories; lane 0 the reference's npz."""
    import torch
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    from oracle import c_oracle
    x_ref, u_ref = load_refs()
    B = 1 << 20
    x0 = make_x0(B)
    eng = AcrobotEngine()
    kw = dict(tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20)
    s = BatchedNewtonSolver(eng, x_ref, u_ref, B, **kw)
    assert s.schedule == "pipelined"
    r = s.solve(x0, 5000, sync_every=4)
    st = r.status.cpu().numpy()
    assert (st == 1).all(), np.bincount(st)
    ni = r.n_iter.cpu().numpy()
    nr, cost = r.n_rollouts.cpu().numpy(), r.cost.cpu().numpy()
    fx = load_golden("headline_oracle")
    L = len(fx["n_iter"])
    np.testing.assert_array_equal(make_x0(L), x0[:L])
    np.testing.assert_array_equal(ni[:L], fx["n_iter"])
    np.testing.assert_array_equal(st[:L], fx["status"])
    np.testing.assert_array_equal(nr[:L], fx["n_rollouts"])
    rel = np.abs(cost[:L] - fx["cost"]) / np.abs(fx["cost"])
    assert rel.max() < 1e-11, rel.max()
    head = {k: getattr(r, k)[:4096].cpu().numpy() for k in ("x", "u", "K", "sigma", "cost")}
    head["n_iter"], head["n_roll"] = ni[:4096], r.n_rollouts[:4096].cpu().numpy()
    pick = np.linspace(0, B - 1, 1024).astype(np.int64)   # ~3 s of the C oracle on the box's host cores
    xs, us = r.x[pick].cpu().numpy(), r.u[pick].cpu().numpy()
    x0l, u0l = r.x[0].cpu().numpy(), r.u[0].cpu().numpy()
    del r, s
    torch.cuda.empty_cache()
    g = load_golden("task2_reference_output")
    assert rel_l2(x0l, g["x"]) < TOL_TRAJ and rel_l2(u0l, g["u"]) < TOL_TRAJ
    o = c_oracle.newton_solve(x0[pick], x_ref, u_ref, max_iters=5000, tol=1e-4, gamma_0=0.1)
    np.testing.assert_array_equal(ni[pick], o["n_iter"])
    assert _lane_rel(xs, o["x"]).max() < TOL_TRAJ and _lane_rel(us, o["u"]).max() < TOL_TRAJ
    r2 = BatchedNewtonSolver(eng, x_ref, u_ref, 4096, **kw).solve(x0[:4096], 5000)
    assert r2.schedule == "persistent"
    np.testing.assert_array_equal(head["n_iter"], r2.n_iter.cpu().numpy())
    np.testing.assert_array_equal(head["n_roll"], r2.n_rollouts.cpu().numpy())
    for k in ("x", "u", "K", "sigma", "cost"):
        np.testing.assert_array_equal(head[k], getattr(r2, k).cpu().numpy(), err_msg=k)


# ----------------------------------------------------------------------------- BASELINE cfg 5
def test_cfg5_full_size_matches_oracle():
    """BASELINE cfg 5 exactly as bench.py --workload mpc runs it: 8,192 disturbed initial states, horizon 50,
    500 control steps, against the numpy restatement (oracle/tracking_np.py) for every lane."""
    from gymnast_optimalcontrol_amd import trajectory_tracking as tt
    from oracle import tracking_np as tr
    g = load_golden("task2_reference_output")
    x_ref, u_ref = g["x"], g["u"]
    B = 8192
    x0 = x_ref[0] + np.random.default_rng(0).uniform(-0.1, 0.1, (B, 4))
    x0[0] = x_ref[0] + 0.1
    x, u, K0 = tt.solve_mpc_tracking_batch(x0, x_ref, u_ref, 50)
    xo, uo, K0o = tr.solve_mpc_tracking(x0, x_ref, u_ref, 50)
    assert x.shape == (B, 501, 4) and u.shape == (B, 500, 2)
    assert np.abs(K0.cpu().numpy() - K0o).max() <= 1e-9 * np.abs(K0o).max()
    ex, eu = _lane_rel(x.cpu().numpy(), xo), _lane_rel(u.cpu().numpy(), uo)
    assert ex.max() < 1e-9 and eu.max() < 1e-9, (ex.max(), eu.max())


# ------------------------------------------------------------------------ parameter sets 2 / 3
@pytest.mark.parametrize("pset", [2, 3])
def test_parameter_sets_on_device(pset):
    """dynamics.py:31-61 parameter sets on the device: the primitives against the reference's own set_params
    lambdified (tests/golden/pset_kats.npz), and a batched solve with the set against both oracles."""
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.params import PARAM_NAMES, PARAM_SETS
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    from oracle import acrobot_np as onp, c_oracle
    from bench import load_refs
    g = load_golden("pset_kats")
    eng = AcrobotEngine(params=pset)
    X, U = g["X"], g["U"]
    np.testing.assert_allclose(eng.continuous_dynamics(X, U).cpu().numpy(), g[f"p{pset}_f_cont"], rtol=1e-11,
                               atol=1e-9)
    np.testing.assert_allclose(eng.rk4(X, U).cpu().numpy(), g[f"p{pset}_f_rk4"], rtol=1e-11, atol=1e-9)
    A, B = eng.jacobians(X, U)
    np.testing.assert_allclose(A.cpu().numpy(), g[f"p{pset}_A_c"], rtol=1e-10, atol=1e-8)
    np.testing.assert_allclose(B.cpu().numpy(), g[f"p{pset}_B_c"], rtol=1e-10, atol=1e-12)

    x_ref, u_ref = load_refs()
    L = 24
    x0 = np.zeros((L, 4)); x0[1:, :2] = np.random.default_rng(pset).uniform(-0.5, 0.5, (L - 1, 2))
    r = BatchedNewtonSolver(eng, x_ref, u_ref, L, tol=1e-4, gamma_0=0.1).solve(x0, 30)
    o = onp.newton_solve(x0, x_ref, u_ref, 30, tol=1e-4, gamma_0=0.1, pset=pset)
    params = tuple(PARAM_SETS[pset][k] for k in PARAM_NAMES)
    oc = c_oracle.newton_solve(x0, x_ref, u_ref, max_iters=30, tol=1e-4, gamma_0=0.1, params=params)
    for ref in (o, oc):
        np.testing.assert_array_equal(r.n_iter.cpu().numpy(), ref["n_iter"])
        np.testing.assert_array_equal(r.status.cpu().numpy(), ref["status"])
        np.testing.assert_array_equal(r.n_rollouts.cpu().numpy(), ref["n_rollouts"])
        assert _lane_rel(r.x.cpu().numpy(), ref["x"]).max() < 1e-9
        assert _lane_rel(r.K.cpu().numpy(), ref["K"]).max() < 1e-8
        np.testing.assert_allclose(r.cost.cpu().numpy(), ref["cost"], rtol=1e-10)
    # a different set gives a different solve (the set really reaches the kernels)
    r1 = BatchedNewtonSolver(AcrobotEngine(), x_ref, u_ref, L, tol=1e-4, gamma_0=0.1).solve(x0, 30)
    assert np.abs(r1.cost.cpu().numpy() - r.cost.cpu().numpy()).max() > 1.0


# ---------------------------------------------------------------- selected-lane trajectory capture
@pytest.mark.parametrize("schedule", ["serial", "pipelined", "persistent"])
def test_capture_lanes_reproduce_reference_history(schedule, task2_refs):
    """capture_lanes: the batched solver's per-lane history['x_trajs'] (trajectory_generation.py:322-327,
    387-388).  Lane 0 is task 2's golden lane: 394 entries (x_0 and one per accepted iteration), the kept ones
    equal to the reference's; a backtracking / failing lane's list has one entry per accepted iteration."""
    from gymnast_optimalcontrol_amd import _lib
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    g = load_golden("task2_solve")
    L = load_golden("lanes")
    xr, ur, _ = task2_refs
    names = list(L["names"])
    fail = names.index("lane_vel_s14")                    # LS failure at iteration 91 (reference)
    x0 = np.zeros((70, 4)); x0[1:, :2] = np.random.default_rng(9).uniform(-0.5, 0.5, (69, 2))
    x0[33] = L["x0"][fail]
    s = BatchedNewtonSolver(AcrobotEngine(), xr, ur, 70, tol=1e-4, gamma_0=0.1, capture_lanes=[0, 33],
                            hist_len=1000, pipeline=schedule == "pipelined", persistent=schedule == "persistent")
    r = s.solve(x0, 5000)
    assert r.schedule == schedule
    # capturing (trajectories, and sigma re-runs at iterations 0-2) leaves the solve bit for bit unchanged
    r_plain = BatchedNewtonSolver(AcrobotEngine(), xr, ur, 70, tol=1e-4, gamma_0=0.1, hist_len=1000,
                                  pipeline=schedule == "pipelined", persistent=schedule == "persistent").solve(x0, 5000)
    for k in ("x", "u", "K", "sigma", "cost", "n_iter", "n_rollouts", "status"):
        assert np.array_equal(getattr(r, k).cpu().numpy(), getattr(r_plain, k).cpu().numpy(), equal_nan=True), k
    tr = r.x_trajs
    assert len(tr[0]) == len(g["cost_hist"]) == 394
    for j, it in enumerate(g["x_hist_idx"]):     # x_0 of the golden lane is the rest state: all zeros
        np.testing.assert_allclose(tr[0][it], g["x_hist"][j], rtol=TOL_TRAJ, atol=1e-12, err_msg=str(it))
    np.testing.assert_array_equal(tr[0][-1], r.x[0].cpu().numpy())
    assert int(r.status[33]) == _lib.LS_FAILED
    assert len(tr[33]) == int(r.n_iter[33])                # x_0 + (n_iter - 1) accepted iterations
    np.testing.assert_array_equal(tr[33][-1], r.x[33].cpu().numpy())
    assert rel_l2(tr[33][-1], L["x"][fail]) < TOL_TRAJ
    # the batched lane feeds the reference's report (main.task_2 -> generate_report_graphs)
    import matplotlib
    matplotlib.use("Agg")
    from gymnast_optimalcontrol_amd import trajectory_generation as tg
    h = tg.lane_history(r, 0)
    np.testing.assert_allclose(h["cost"], g["cost_hist"], rtol=1e-9)
    np.testing.assert_allclose(h["sigma_norm"], g["sigma_norm_hist"], rtol=1e-6)
    # history['sigmas'] (:341): the reference's length, sigma at the iterations its report plots (:476-480)
    assert len(h["sigmas"]) == 393 and sorted(r.sigmas[0]) == [0, 1, 2]
    assert rel_l2(h["sigmas"][0], g["sigma_first"]) < 1e-8
    assert rel_l2(h["sigmas"][392], g["sigma"]) < 1e-6
    assert all(h["sigmas"][i] is None for i in range(3, 392))
    # the lane that fails the line search: sigma of its iterations 0-2 and of its last (failed) iteration
    hf = tg.lane_history(r, 33)
    assert len(hf["sigmas"]) == int(r.n_iter[33]) and sorted(r.sigmas[33]) == [0, 1, 2]
    d = tg.generate_report_graphs(g["t_ref"], g["x_ref"], g["u_ref"], r.x[0].cpu().numpy(), r.u[0].cpu().numpy(), h)
    assert d["iterations_shown"][-1] == 393 and len(d["figures"]) == 4
    assert d["sigma_iterations"] == [0, 1, 2, 392]
    np.testing.assert_array_equal(d["sigma_tau2"][392], r.sigma[0, :, 1].cpu().numpy())
    import matplotlib.pyplot as plt
    plt.close("all")


# ------------------------------------------------------------------ sharded solve on the HIP path
@pytest.mark.parametrize("total", [301, 32769])
def test_sharded_solve_on_hip_matches_unsharded(total, tmp_path):
    """Two ranks (gloo, sharing this GPU) run distributed.solve_sharded on the HIP solver.  32,769 lanes give
    ragged shards of 16,385 / 16,384 lanes on either side of the persistent-schedule threshold (64 lanes per CU
    on 256 CUs): both ranks must still pick the same schedule (chosen on the largest shard), pair up their
    all-reduces, and reproduce the unsharded solve bit for bit; 301 lanes run the persistent schedule.  With 32,769
    lanes the worker also solves 2,000 hard lanes with lane compaction forced (rank-local) and the straggler tail
    (switched on the global count): gathered, the unsharded solve's bits."""
    import torch
    from bench import load_refs
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from sharded_worker import sharded_x0
    max_iters = 600
    out = str(tmp_path / "shard")
    env = dict(os.environ, GYM_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    port = 29500 + (os.getpid() % 1000) + (total % 97)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "tests", "sharded_worker.py"),
           out, str(total), str(max_iters), "7"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    parts = [np.load(f"{out}.rank{r}.npz") for r in range(2)]
    assert str(parts[0]["schedule"]) == str(parts[1]["schedule"])
    assert (int(parts[0]["hi"]) - int(parts[0]["lo"])) - (int(parts[1]["hi"]) - int(parts[1]["lo"])) == total % 2
    # the global stop: both ranks read the same all-reduced statistics
    np.testing.assert_array_equal(parts[0]["stats"], parts[1]["stats"])
    x_ref, u_ref = load_refs()
    x0 = sharded_x0(total, 7)
    s = BatchedNewtonSolver(AcrobotEngine(), x_ref, u_ref, total, tol=1e-4, gamma_0=0.1)
    r = s.solve(x0, max_iters)
    full = {k: getattr(r, k).cpu().numpy() for k in ("x", "u", "K", "sigma", "cost", "n_iter", "status",
                                                      "n_rollouts")}
    for rk in range(2):                  # distributed.gather_sharded: the global per-lane results on every rank
        g = np.load(f"{out}.gathered.rank{rk}.npz")
        for k in ("cost", "n_iter", "status"):
            np.testing.assert_array_equal(g[k], full[k], err_msg=f"gathered {k} on rank {rk}")
    for p_ in parts:
        lo, hi = int(p_["lo"]), int(p_["hi"])
        for k, v in full.items():
            assert np.array_equal(p_[k], v[lo:hi], equal_nan=True), (k, lo, hi)
    assert (full["n_rollouts"] > full["n_iter"]).any()        # some lanes backtracked
    # per-lane references cut to each rank's shard (sharded_worker.py): bit for bit the unsharded per-lane solve
    xr3 = np.broadcast_to(x_ref, (total,) + x_ref.shape).copy()
    ur3 = np.broadcast_to(u_ref, (total,) + u_ref.shape).copy()
    ur3[1::3, :, 1] *= 0.8
    r3 = BatchedNewtonSolver(AcrobotEngine(), xr3, ur3, total, tol=1e-4, gamma_0=0.1).solve(x0, 40)
    for rk in range(2):
        p3 = np.load(f"{out}.perlane.rank{rk}.npz")
        lo, hi = int(p3["lo"]), int(p3["hi"])
        for k in ("x", "cost", "n_iter"):
            assert np.array_equal(p3[k], getattr(r3, k)[lo:hi].cpu().numpy(), equal_nan=True), (k, rk)
    if total > 1000:   # hard lanes, lane compaction forced on each rank, the straggler tail: the unsharded solve's bits
        from sharded_worker import hard_x0
        xh = hard_x0(2000, 3)
        rh = BatchedNewtonSolver(AcrobotEngine(), x_ref, u_ref, 2000, tol=1e-4, gamma_0=0.1, compact=False,
                                 tail_lanes=0, hist_len=200).solve(xh, 200)
        assert (rh.n_rollouts > rh.n_iter).sum() > 10
        for rk in range(2):
            gh = np.load(f"{out}.hard.rank{rk}.npz")
            for k in ("x", "u", "K", "sigma", "cost", "n_iter", "status", "n_rollouts", "gamma"):
                assert np.array_equal(gh[k], getattr(rh, k).cpu().numpy(), equal_nan=True), ("hard", k, rk)
    torch.cuda.synchronize()


# ------------------------------------------------------------------ the RCCL branch on one GPU
def test_rccl_collectives_on_one_gpu(tmp_path):
    """The device-tensor RCCL branches of distributed.py, executed before the driver's 8-GPU run does: a 1-rank
    group on backend "nccl" (with device_id), solve_sharded(gather=True, force_collectives=True) on the
    persistent, pipelined and serial schedules, max_over_ranks / sum_over_ranks, and per-lane references cut to
    the shard.  Every all-reduce is on a fp64 device tensor enqueued from the solver's stream, every result field
    is all-gathered on the device, and the gathered results are bit for bit the plain solve's (tests/rccl_worker.py
    checks; it runs in its own process so the process group cannot leak into other tests)."""
    import json
    out = tmp_path / "rccl.json"
    env = dict(os.environ)
    env.pop("GYM_DIST_BACKEND", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_worker.py"), str(out), "301", "600"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    s = json.loads(out.read_text())
    assert s["backend"] == "nccl" and s["world_size"] == 1
    assert set(s["schedules"]) == {"persistent", "pipelined", "serial"}
    for sched, d in s["schedules"].items():
        assert d["all_reduce_calls"] >= 1 and d["all_gather_calls"] == 9, (sched, d)
        assert d["backtracked"] > 0                      # the wide-start lanes exercise the retry path too


# ------------------------------------------------------------------ bench.py --gpus N without a launcher
def test_bench_spawns_ranks_on_the_gpu():
    """bench.py --gpus 2 with no launcher starts two ranks itself (gloo: both share this GPU; RCCL refuses two
    ranks on one device): the line reports n_gpus 2, a 2-rank process group and twice the lanes; rank 0's shard
    is the N = 1 workload, so lane 0's parity record and the per-GPU lane count equal the single-process line's."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["GYM_DIST_BACKEND"] = "gloo"
    args = ["--batch", "512", "--steps", "1", "--warmup", "0", "--no-cpu", "--extra-legs", ""]

    def line(n):
        p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), *args], env=env,
                           capture_output=True, text=True, timeout=280)
        assert p.returncode == 0, p.stderr[-3000:]
        return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])

    two, one = line(2), line(1)
    assert two["n_gpus"] == 2 and two["dist"]["world_size"] == 2 and two["dist"]["backend"] == "gloo"
    assert two["dist"]["launcher"] == "bench.py (spawned ranks)"
    assert one["n_gpus"] == 1 and one["dist"]["world_size"] == 1
    assert two["config"]["global_lanes"] == 1024 and two["config"]["lanes_per_gpu"] == 512
    assert one["config"]["global_lanes"] == one["config"]["lanes_per_gpu"] == 512
    for k in ("lane0_iters", "lane0_rel_l2_x", "lane_iters_min_max"):
        assert two["parity"][k] == one["parity"][k], k
    assert two["value"] > 0 and two["scaling"] == "weak"
    # per-rank diagnostics: each rank's own elapsed time (the slowest one is the line's time, up to the closing
    # barrier), lane-iterations summing to the job's, and the statistics all-reduce's host time
    d = two["dist"]
    el = d["rank_elapsed_s"]
    assert len(el) == 2 and d["rank_elapsed_min_max"] == [min(el), max(el)]
    total_s = two["ms_per_step"] * two["steps"] / 1e3
    assert max(el) <= total_s + 1e-6 and max(el) > 0.9 * total_s, (el, total_s)
    lanes = d["rank_lane_iterations"]
    assert len(lanes) == 2 and abs(sum(lanes) - two["value"] * total_s) <= 1 and min(lanes) > 0
    assert d["allreduce_calls_per_step"] > 0 and d["allreduce_8xf64_us"] > 0
    assert all(0 <= t < total_s for t in d["rank_reduce_host_s"] + d["rank_readback_host_s"])
    assert "rank_elapsed_s" not in one["dist"]


def test_kernel_timing_covers_every_launch():
    """bench.py's roofline divides the algorithmic bytes by the phase kernel's average HIP-event time: every launch
    between two host synchronisations is timed (GYM_TIMING_POOL), not a sample, on the pipelined and the persistent
    schedules."""
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    x_ref, u_ref = load_refs()
    eng = AcrobotEngine()
    for kw, kinds, key in ((dict(pipeline=True), ("phase_odd", "phase_even"), "phase"),
                           (dict(persistent=True, chunk=16), ("run",), "run")):
        s = BatchedNewtonSolver(eng, x_ref, u_ref, 4096, tol=1e-4, gamma_0=0.1, **kw).enable_timing()
        s.solve(make_x0(4096), 60, sync_every=4)
        s.reset_timing()
        s.solve(make_x0(4096), 60, sync_every=4)
        kt = s.kernel_times()
        assert sum(kt[k][1] for k in kinds) == s.launches[key] > 0, (kt, s.launches)
        assert all(kt[k][0] > 0 for k in kinds)
