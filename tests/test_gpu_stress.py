"""Hard lanes at scale: SURVEY 8(d)'s stress distribution through the AUTOMATIC schedule (pipelined, lane
compaction, the low-occupancy regime, the straggler tail), decision by decision against the C oracle, and on
selected lanes against the reference's own newton_Algorithm, through the C-ABI.

Far from convergence and at the stall that ends an Armijo failure, the line search compares costs that agree to
rounding: J_new - (J + c gamma dJ) is then ~1e-14 |J| (trajectory_generation.py:361), and two restatements that
round differently (the GPU's closed forms, the C oracle's, the reference's sympy / LAPACK) may take such a test
either way.  The contract checked here, lane by lane (tests/stress_settle.py):
  * a lane without any Armijo test within 1e-11 of a tie (the oracle's record) has exactly the oracle's decisions;
  * every lane whose decisions (iteration count, status, rollout count) differ from the oracle's is re-run with
    per-iteration records on both sides, and the FIRST iteration at which they part (the Armijo trial count, or the
    cost after it) carries an oracle Armijo margin below TIE = 3e-12 at that very iteration (a tie both sides took
    the same way earlier does not count), or a convergence test within 1e-9 of tol;
  * on the reference-run lanes (tests/golden/make_golden_stress.py), where the reference's own record has no tie the
    GPU takes the reference's decisions exactly, and where the GPU and the oracle part the reference's record shows a
    tie at or before that point.
No tolerance on decisions is loosened: every difference is attributed to a tie at the iteration it happens.
"""
import numpy as np
import pytest

from conftest import load_golden
from stress_settle import COST_REL, assert_settled, oracle_record, settle

pytestmark = pytest.mark.gpu

TIE_FIXTURE = 1e-11   # the fixtures' k_tie / margin_min threshold (tests/golden/make_stress_oracle.py: TIE)


def _hard_x0(B=2048, seed=7):
    """tools/stress_parity.py's hard set: th ~ U(+-1.5), every 4th lane with thdot ~ U(+-2)."""
    rng = np.random.default_rng(seed)
    x0 = np.zeros((B, 4))
    x0[:, :2] = rng.uniform(-1.5, 1.5, (B, 2))
    x0[::4, 2:] = rng.uniform(-2.0, 2.0, (len(x0[::4]), 2))
    return x0


def _decisions(r):
    return r.n_iter.cpu().numpy(), r.status.cpu().numpy(), r.n_rollouts.cpu().numpy()


def test_stress_batch_decisions_vs_oracle():
    """bench.py's stress workload exactly as `bench.py --workload stress` (and the line's stress leg) runs it:
    262,144 lanes, th ~ U(+-1.5), the automatic schedule with every regime engaged, against the C oracle's outcome for
    every lane (tests/golden/stress_oracle.npz); then EVERY differing lane settled at the iteration it parts."""
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
    assert float(o["tie"]) == TIE_FIXTURE
    no, so, ro, co, k_tie = (o[k] for k in ("n_iter", "status", "n_rollouts", "cost", "k_tie"))
    same = (ng == no) & (sg == so) & (rg == ro)
    # every lane without a tie anywhere in the oracle's record has exactly the oracle's decisions
    assert same[k_tie < 0].all()
    conv = same & (so == _lib.CONVERGED)
    assert np.max(np.abs(cg[conv] - co[conv]) / np.abs(co[conv])) < 1e-11
    assert conv.sum() > 0.8 * B and (so == _lib.LS_FAILED).sum() > 0.1 * B
    # every differing lane: both sides' per-iteration records, the tie at the iteration they part
    diff = np.nonzero(~same)[0]
    d = settle(eng, x0, xr, ur, diff)
    assert_settled(d, ng[diff], sg[diff], rg[diff])
    print(f"{len(diff)} differing lanes settled; margins at the divergence: max {d['margin_k'].max():.3e}, "
          f"< 1e-13: {int((d['margin_k'] < 1e-13).sum())}, kinds {dict(zip(*np.unique(d['kind'], return_counts=True)))}")


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
    xr, ur = load_refs()
    x0 = _hard_x0()
    B, H = len(x0), 5000
    eng = AcrobotEngine()
    s = BatchedNewtonSolver(eng, xr, ur, B, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20, hist_len=H,
                            schedule_lanes=262144, tail_lanes=128)
    r = s.solve(x0, H, sync_every=4)
    assert r.schedule == "pipelined" and r.compactions > 0
    assert r.lowocc_lane_iterations > 0 and r.tail_lane_iterations > 0
    o = oracle_record(x0, xr, ur)
    ng, sg, rg = _decisions(r)
    same = (ng == o["n_iter"]) & (sg == o["status"]) & (rg == o["n_rollouts"])
    diff = np.nonzero(~same)[0]
    assert_settled(settle(eng, x0, xr, ur, diff), ng[diff], sg[diff], rg[diff])
    tie_free = ~(np.nanmin(np.where(np.isnan(o["hist_margin"]), np.inf, o["hist_margin"]), axis=1) < TIE_FIXTURE)
    assert same[tie_free].all()
    conv = same & (o["status"] == _lib.CONVERGED)
    assert conv.sum() > B // 2 and (o["status"] == _lib.LS_FAILED).sum() > 50
    xg = r.x.cpu().numpy()[conv]
    ex = np.linalg.norm((xg - o["x"][conv]).reshape(conv.sum(), -1), axis=1) / \
        np.linalg.norm(o["x"][conv].reshape(conv.sum(), -1), axis=1)
    assert ex.max() < 1e-8, ex.max()
    cg = r.cost.cpu().numpy()
    assert np.max(np.abs(cg[conv] - o["cost"][conv]) / np.abs(o["cost"][conv])) < 1e-11


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
    eng = AcrobotEngine()
    s = BatchedNewtonSolver(eng, xr, ur, B, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20,
                            hist_len=H, schedule_lanes=262144, tail_lanes=128)
    r = s.solve(x0, H, sync_every=4)
    assert r.schedule == "pipelined" and r.tail_lane_iterations > 0
    o = oracle_record(x0, xr, ur)
    ng, sg, rg = _decisions(r)
    same = (ng == o["n_iter"]) & (sg == o["status"]) & (rg == o["n_rollouts"])
    diff = np.nonzero(~same)[0]
    assert_settled(settle(eng, x0, xr, ur, diff), ng[diff], sg[diff], rg[diff])
    tie_free = ~(np.nanmin(np.where(np.isnan(o["hist_margin"]), np.inf, o["hist_margin"]), axis=1) < TIE_FIXTURE)
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
    has one (within 1e-11: the reference's record holds costs, not trial counts, so the iteration a trial flips is
    not located on it), the GPU's cost history equals the reference's until the reference's first tie."""
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
        if not (np.nanmin(mref) < TIE_FIXTURE):
            assert (ng[j], sg[j], rg[j]) == (nr, g["status"][j], g["n_rollouts"][j]), int(lane)
            continue
        k_tie = int(np.argmax(mref < TIE_FIXTURE))
        n = min(k_tie, int(ng[j]))
        rel = np.abs(hg[j, :n] - href[:n]) / np.abs(href[:n])
        assert (rel <= COST_REL).all(), (int(lane), k_tie, float(np.nanmax(rel)))


def test_stress_tie_lanes_vs_reference():
    """TIE (3e-12) pinned to the reference itself.  tests/golden/stress_tie_lanes.npz holds the
    reference's newton_Algorithm run (make_golden_stress_ties.py) on the 58 stress lanes whose GPU / C-oracle divergence
    has the largest oracle margins (>= 1e-13 at the iteration k where they part, the five above 1e-12 included), each
    to iteration k, with its per-iteration trial counts and Armijo margins.  The GPU's per-iteration record on the same
    lanes (serial schedule, bitwise every schedule) must follow the reference's decisions through k, or part from the
    reference at an iteration where the reference's own margin is below TIE: no GPU decision differs from the
    reference's except at a tie of the reference's own record."""
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from stress_settle import TIE, gpu_record
    g = load_golden("stress_tie_lanes")
    lanes, kdiv = g["lanes"], g["k"]
    x0 = make_x0(262144, spread=1.5)[lanes]
    xr, ur = load_refs()
    _, _, _, tg, _, _ = gpu_record(AcrobotEngine(), x0, xr, ur, max_iters=int(kdiv.max()) + 1)
    sided, tied = [], []
    for j, lane in enumerate(lanes):
        n = int(g["n_iter"][j])                       # the reference ran iterations 0 .. k
        assert n == int(kdiv[j]) + 1
        rt, rm = g["trials"][j, :n], g["margin"][j, :n]
        diff = np.nonzero(tg[j, :n] != rt)[0]
        if len(diff) == 0:
            sided.append(int(lane))                   # the GPU takes the reference's decision at k (and before)
            continue
        kd = int(diff[0])
        assert rm[kd] < TIE, (int(lane), kd, int(kdiv[j]), float(rm[kd]), int(tg[j, kd]), int(rt[kd]))
        tied.append((int(lane), kd))
    print(f"{len(sided)} lanes take the reference's decisions through k; {len(tied)} part from it at a reference tie")
    assert len(sided) + len(tied) == len(lanes)
