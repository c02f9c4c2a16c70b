"""Hard lanes at scale: SURVEY 8(d)'s stress distribution through the AUTOMATIC schedule (pipelined, lane
compaction, the low-occupancy regime, the straggler tail), decision by decision against the C oracle, and on
selected lanes against the reference's own newton_Algorithm, through the C-ABI.

Far from convergence and at the stall that ends an Armijo failure, the line search compares costs that agree to
rounding: J_new - (J + c gamma dJ) is then ~1e-14 |J| (trajectory_generation.py:361), and two restatements that
round differently (the GPU's closed forms, the C oracle's, the reference's sympy / LAPACK) may take such a test
either way.  The contract checked here:
  * a lane whose decisions (iteration count, status, rollout count) differ from the oracle's had an Armijo test within
    TIE (1e-11) of a tie before either run ended (the oracle's per-iteration record, oracle/c_oracle.py hist_margin),
    and, where histories are compared, its cost history agrees with the oracle's until that tie;
  * a lane without any such tie has exactly the oracle's decisions; converged lanes' costs agree to 1e-11;
  * on the reference-run lanes (tests/golden/make_golden_stress.py), where the reference's own record has no tie the
    GPU takes the reference's decisions exactly, and where the GPU and the oracle part the reference's record shows a
    tie at or before that point.
No tolerance on decisions is loosened: every difference is attributed to a recorded tie.
"""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

TIE = 1e-11          # relative Armijo margin counted as a tie (tests/golden/make_stress_oracle.py: TIE)
COST_REL = 1e-9      # cost histories "agree" (pre-tie differences are ~1e-13)


def _hard_x0(B=2048, seed=7):
    """tools/stress_parity.py's hard set: th ~ U(+-1.5), every 4th lane with thdot ~ U(+-2)."""
    rng = np.random.default_rng(seed)
    x0 = np.zeros((B, 4))
    x0[:, :2] = rng.uniform(-1.5, 1.5, (B, 2))
    x0[::4, 2:] = rng.uniform(-2.0, 2.0, (len(x0[::4]), 2))
    return x0


def _decisions(r):
    return r.n_iter.cpu().numpy(), r.status.cpu().numpy(), r.n_rollouts.cpu().numpy()


def _first_divergence(hg, ho, ng, no):
    """First iteration whose cost (after it) differs by more than COST_REL between the two records, or the first
    iteration only one of the runs executed."""
    n = min(ng, no)
    a, b = hg[:n], ho[:n]
    rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    both_nan = np.isnan(a) & np.isnan(b)                   # a failed iteration on both sides: no cost after it
    bad = np.nonzero(~((rel <= COST_REL) | both_nan))[0]
    return int(bad[0]) if len(bad) else n


def _settle_with_histories(x0, xr, ur, lanes_gpu_solver, idx):
    """Re-run lanes ``idx`` on the GPU with per-lane histories (lanes are independent: every schedule gives each
    lane the same bits at any batch size) and on the C oracle with its record; every lane's first divergence must
    come at or after an oracle Armijo test within TIE of a tie.  Returns the number of lanes checked."""
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    from oracle import c_oracle
    eng = lanes_gpu_solver
    H = 5000
    s = BatchedNewtonSolver(eng, xr, ur, len(idx), tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20, hist_len=H)
    r = s.solve(x0[idx], H)
    o = c_oracle.newton_solve(x0[idx], xr, ur, max_iters=H, tol=1e-4, gamma_0=0.1, hist_len=H)
    ng, _, _ = _decisions(r)
    hg = r.hist_cost.cpu().numpy().T
    for j in range(len(idx)):
        k = _first_divergence(hg[j], o["hist_cost"][j], int(ng[j]), int(o["n_iter"][j]))
        m = o["hist_margin"][j, :k + 1]
        assert np.nanmin(m) < TIE, (int(idx[j]), k, float(np.nanmin(m)))
    return len(idx)


def test_stress_batch_decisions_vs_oracle():
    """bench.py's stress workload exactly as `bench.py --workload stress` (and the line's stress leg) runs it:
    262,144 lanes, th ~ U(+-1.5), the automatic schedule with every regime engaged, against the C oracle's outcome for
    every lane (tests/golden/stress_oracle.npz)."""
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd import _lib
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr, ur = load_refs()
    B = 262144
    x0 = make_x0(B, spread=1.5)
    eng = AcrobotEngine()
    s = BatchedNewtonSolver(eng, xr, ur, B, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20)
    r = s.solve(x0, 5000, sync_every=4)
    assert r.schedule == "pipelined" and r.compactions > 0
    assert r.lowocc_lane_iterations > 0 and r.tail_lane_iterations > 0       # every regime engaged
    ng, sg, rg = _decisions(r)
    cg = r.cost.cpu().numpy()
    del r, s
    o = load_golden("stress_oracle")
    assert float(o["tie"]) == TIE
    no, so, ro, co, k_tie = (o[k] for k in ("n_iter", "status", "n_rollouts", "cost", "k_tie"))
    same = (ng == no) & (sg == so) & (rg == ro)
    diff = np.nonzero(~same)[0]
    # every differing lane had an Armijo test within TIE of a tie before either run ended ...
    unexplained = diff[~((k_tie[diff] >= 0) & (k_tie[diff] < np.minimum(ng[diff], no[diff])))]
    assert len(unexplained) == 0, (len(unexplained), unexplained[:10])
    # ... and every lane without one has exactly the oracle's decisions
    assert same[k_tie < 0].all()
    conv = same & (so == _lib.CONVERGED)
    assert np.max(np.abs(cg[conv] - co[conv]) / np.abs(co[conv])) < 1e-11
    assert conv.sum() > 0.8 * B and (so == _lib.LS_FAILED).sum() > 0.1 * B
    # the divergence of a sample of differing lanes, pinned on both sides' histories
    pick = diff[np.linspace(0, len(diff) - 1, min(len(diff), 48)).astype(np.int64)]
    assert _settle_with_histories(x0, xr, ur, eng, pick) == len(pick)


def test_stress_hard_lanes_vs_live_oracle():
    """2,048 hard lanes (th ~ U(+-1.5), every 4th with thdot ~ U(+-2)) through the automatic schedule of a
    262,144-lane shard (schedule_lanes) with the tail at 128 lanes, so that the pipelined schedule compacts, enters
    the low-occupancy regime and hands the last lanes to the tail, against the C oracle run beside it with its
    per-iteration record: decisions, costs and trajectories of the agreeing lanes, every other lane settled by a
    tie before its first divergence."""
    from bench import load_refs
    from gymnast_optimalcontrol_amd import _lib
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    from oracle import c_oracle
    xr, ur = load_refs()
    x0 = _hard_x0()
    B, H = len(x0), 5000
    eng = AcrobotEngine()
    s = BatchedNewtonSolver(eng, xr, ur, B, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20, hist_len=H,
                            schedule_lanes=262144, tail_lanes=128)
    r = s.solve(x0, H, sync_every=4)
    assert r.schedule == "pipelined" and r.compactions > 0
    assert r.lowocc_lane_iterations > 0 and r.tail_lane_iterations > 0
    o = c_oracle.newton_solve(x0, xr, ur, max_iters=H, tol=1e-4, gamma_0=0.1, hist_len=H)
    ng, sg, rg = _decisions(r)
    same = (ng == o["n_iter"]) & (sg == o["status"]) & (rg == o["n_rollouts"])
    hg = r.hist_cost.cpu().numpy().T
    for l in np.nonzero(~same)[0]:
        k = _first_divergence(hg[l], o["hist_cost"][l], int(ng[l]), int(o["n_iter"][l]))
        assert np.nanmin(o["hist_margin"][l, :k + 1]) < TIE, (int(l), k)
    tie_free = ~(np.nanmin(np.where(np.isnan(o["hist_margin"]), np.inf, o["hist_margin"]), axis=1) < TIE)
    assert same[tie_free].all()
    conv = same & (o["status"] == _lib.CONVERGED)
    assert conv.sum() > B // 2 and (o["status"] == _lib.LS_FAILED).sum() > 50
    xg = r.x.cpu().numpy()[conv]
    ex = np.linalg.norm((xg - o["x"][conv]).reshape(conv.sum(), -1), axis=1) / \
        np.linalg.norm(o["x"][conv].reshape(conv.sum(), -1), axis=1)
    assert ex.max() < 1e-8, ex.max()
    cg = r.cost.cpu().numpy()
    assert np.max(np.abs(cg[conv] - o["cost"][conv]) / np.abs(o["cost"][conv])) < 1e-11


def _oracle_groups(x0, xr, ur, H):
    """The C oracle (shared references only) over per-lane references: one run per distinct reference, merged."""
    from oracle import c_oracle
    if xr.ndim == 2:
        return c_oracle.newton_solve(x0, xr, ur, max_iters=H, tol=1e-4, gamma_0=0.1, hist_len=H)
    keys = [ur[l].tobytes() + xr[l].tobytes() for l in range(len(x0))]
    out = None
    for key in dict.fromkeys(keys):
        idx = np.array([l for l, k in enumerate(keys) if k == key])
        o = c_oracle.newton_solve(x0[idx], xr[idx[0]], ur[idx[0]], max_iters=H, tol=1e-4, gamma_0=0.1, hist_len=H)
        if out is None:
            out = {k: np.empty((len(x0),) + v.shape[1:], v.dtype) for k, v in o.items()}
        for k, v in o.items():
            out[k][idx] = v
    return out


@pytest.mark.parametrize("kind", ["task1", "per_lane"])
def test_stress_general_paths_vs_live_oracle(kind):
    """The same contract on the paths the headline does not take: task 1's live tau1 channel (the general,
    tau1-streaming kernels; tests/golden task1_solve's references) and per-lane references (every third lane's
    u_ref scaled by 0.8; the oracle runs each distinct reference separately), 2,048 hard lanes through the automatic
    schedule of a 262,144-lane shard with the tail at 128 lanes."""
    from gymnast_optimalcontrol_amd import _lib
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    x0 = _hard_x0()
    B, H = len(x0), 5000
    if kind == "task1":
        g = load_golden("task1_solve")
        xr, ur = g["x_ref"], g["u_ref_full"]
        assert np.abs(ur[:, 0]).max() > 0                                   # the live tau1 channel
    else:
        from bench import load_refs
        xr, ur = load_refs()
        xr = np.broadcast_to(xr, (B,) + xr.shape).copy()
        ur = np.broadcast_to(ur, (B,) + ur.shape).copy()
        ur[1::3, :, 1] *= 0.8
    s = BatchedNewtonSolver(AcrobotEngine(), xr, ur, B, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20,
                            hist_len=H, schedule_lanes=262144, tail_lanes=128)
    r = s.solve(x0, H, sync_every=4)
    assert r.schedule == "pipelined" and r.tail_lane_iterations > 0
    o = _oracle_groups(x0, xr, ur, H)
    ng, sg, rg = _decisions(r)
    same = (ng == o["n_iter"]) & (sg == o["status"]) & (rg == o["n_rollouts"])
    hg = r.hist_cost.cpu().numpy().T
    for l in np.nonzero(~same)[0]:
        k = _first_divergence(hg[l], o["hist_cost"][l], int(ng[l]), int(o["n_iter"][l]))
        assert np.nanmin(o["hist_margin"][l, :k + 1]) < TIE, (int(l), k)
    tie_free = ~(np.nanmin(np.where(np.isnan(o["hist_margin"]), np.inf, o["hist_margin"]), axis=1) < TIE)
    assert tie_free.sum() > B // 4 and same[tie_free].all()
    conv = same & (o["status"] == _lib.CONVERGED)
    assert conv.sum() > 20 and (o["status"] == _lib.LS_FAILED).sum() > 50
    xg = r.x.cpu().numpy()[conv]
    ex = np.linalg.norm((xg - o["x"][conv]).reshape(conv.sum(), -1), axis=1) / \
        np.linalg.norm(o["x"][conv].reshape(conv.sum(), -1), axis=1)
    assert ex.max() < 1e-8, ex.max()
    cg = r.cost.cpu().numpy()
    assert np.max(np.abs(cg[conv] - o["cost"][conv]) / np.abs(o["cost"][conv])) < 1e-11
    print(kind, "regimes: compactions", r.compactions, "lowocc", r.lowocc_lane_iterations, "tail",
          r.tail_lane_iterations, "same", int(same.sum()), "tie-free", int(tie_free.sum()),
          "statuses", np.bincount(o["status"]))


def test_stress_lanes_vs_reference():
    """The reference's own newton_Algorithm on 27 stress lanes (tests/golden/stress_ref_lanes.npz: every lane whose
    status differs between the GPU and the oracle, 12 lanes whose counts differ, 6 LS-failure and 4 converged lanes
    on which they agree): where the reference's record has no tie, the GPU's decisions are the reference's; where it
    has one, the GPU's cost history equals the reference's until the reference's first tie."""
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    g = load_golden("stress_ref_lanes")
    lanes = g["lanes"]
    x0 = make_x0(262144, spread=1.5)[lanes]
    np.testing.assert_array_equal(x0, g["x0"])
    xr, ur = load_refs()
    H = 5000
    r = BatchedNewtonSolver(AcrobotEngine(), xr, ur, len(lanes), tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20,
                            hist_len=H).solve(x0, H)
    ng, sg, rg = _decisions(r)
    hg = r.hist_cost.cpu().numpy().T
    for j, lane in enumerate(lanes):
        nr = int(g["n_iter"][j])
        mref = g["margin"][j, :nr]
        href = g["cost"][j, 1:]                                  # J after each accepted iteration
        if not (np.nanmin(mref) < TIE):
            assert (ng[j], sg[j], rg[j]) == (nr, g["status"][j], g["n_rollouts"][j]), int(lane)
            continue
        k_tie = int(np.argmax(mref < TIE))
        n = min(k_tie, int(ng[j]))
        rel = np.abs(hg[j, :n] - href[:n]) / np.abs(href[:n])
        assert (rel <= COST_REL).all(), (int(lane), k_tie, float(np.nanmax(rel)))
