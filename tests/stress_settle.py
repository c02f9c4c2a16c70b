"""Per-lane settlement of GPU / C-oracle decision differences on hard lanes (test helper, not a test module).

Far from convergence, and at the stall that ends an Armijo failure, the strict Armijo test of
trajectory_generation.py:361 (J_new < J + c gamma dJ) compares costs equal to rounding, and two restatements that
round differently can take it either way.  For each given lane this runs the GPU solve iteration by iteration on
the serial schedule (bitwise every other schedule: tests/test_gpu_tail.py, test_gpu_parity.py), recording after
each iteration the lane's rollout count, cost and max|sigma| (hist_len), and the C oracle with its per-iteration
record (oracle/c_oracle.py: hist_trials, hist_cost, hist_smax, and hist_margin = the iteration's tightest Armijo
test, min over its trials of |J_new - (J + c gamma dJ)| / |J|).  The first iteration k at which the records part:
  * "trials": iteration k evaluated a different number of Armijo trials on the two sides (a trial accepted on one
    side and rejected on the other; near a stall the two candidates' costs can agree to 1e-12, so the cost record
    alone does not show it), or one side failed the line search there;
  * "cost": the cost after iteration k differs by more than COST_REL with the same trial count: the line search's
    last trial (max_ls) accepted on one side and failed on the other (a NaN cost on that side);
  * "length": every iteration both ran agrees and one run stops first, at the convergence test max|sigma_k| < tol
    (trajectory_generation.py:389-391) taken differently: |max|sigma_k| - tol| / tol is then at rounding level.
For "trials" and "cost" the flipped test is one of iteration k's, so the oracle's own margin at k must be a tie
(margin_k < TIE): a tie at an earlier iteration that both sides took the same way does not explain the lane.
"""
import numpy as np

COST_REL = 1e-9      # cost records "agree" (with the same decisions they differ by up to ~7e-10 on these lanes)
TIE = 3e-12          # an Armijo margin at rounding level: the largest of bench.py's stress batch is 2.80e-12
SMAX_TIE = 1e-9      # max|sigma| at rounding distance from tol (a convergence test taken differently)
H = 5000


def gpu_record(eng, x0, xr, ur, tol=1e-4, max_iters=H):
    """The GPU's per-iteration record of every lane of x0, iteration by iteration on the serial schedule (no tail,
    no compaction, no lane reordering): (n_iter, status, n_rollouts, trials (B, max_iters), cost (B, max_iters),
    smax (B, max_iters)); trials[l, k] = Armijo trials lane l evaluated in iteration k (0 past its last)."""
    import torch
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    B = len(x0)
    s = BatchedNewtonSolver(eng, xr, ur, B, tol=tol, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20, hist_len=max_iters,
                            pipeline=False, persistent=False, tail_lanes=0, compact=False, reorder=False)
    s.max_iters = max_iters
    s.init(x0)
    roll = torch.zeros((max_iters, B), dtype=torch.int32, device=s.n_roll.device)
    for k in range(max_iters):
        st = s.iteration()
        roll[k] = s.n_roll[:B]
        if (k + 1) % 32 == 0 and float(st[0].item()) == 0.0:
            roll[k + 1:] = s.n_roll[:B]
            break
    roll = roll.cpu().numpy().T.astype(np.int64)
    trials = np.diff(roll, axis=1, prepend=0)
    return (s.n_iter[:B].cpu().numpy(), s.status[:B].cpu().numpy(), s.n_roll[:B].cpu().numpy(), trials,
            s.hist_cost[:, :B].cpu().numpy().T, s.hist_smax[:, :B].cpu().numpy().T)


def first_divergence(tg, to, hg, ho, ng, no):
    """(k, kind) of two per-iteration records (trials, cost after the iteration) of one lane; see the module doc."""
    n = min(ng, no)
    bad_t = np.nonzero(tg[:n] != to[:n])[0]
    a, b = hg[:n], ho[:n]
    rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    both_nan = np.isnan(a) & np.isnan(b)                   # a failed iteration on both sides: no cost after it
    bad_c = np.nonzero(~((rel <= COST_REL) | both_nan))[0]
    kt = int(bad_t[0]) if len(bad_t) else n
    kc = int(bad_c[0]) if len(bad_c) else n
    if kt < n and kt <= kc:
        return kt, "trials"
    if kc < n:
        return kc, "cost"
    return n, "length"


def oracle_record(x0, xr, ur, tol=1e-4, max_iters=H):
    """The C oracle with its per-iteration record; per-lane references (xr (B,N,4), ur (B,T,2)) are run one distinct
    reference at a time (the oracle takes a shared reference) and merged."""
    from oracle import c_oracle
    if np.ndim(xr) == 2:
        return c_oracle.newton_solve(x0, xr, ur, max_iters=max_iters, tol=tol, gamma_0=0.1, hist_len=max_iters)
    keys = [ur[l].tobytes() + xr[l].tobytes() for l in range(len(x0))]
    out = None
    for key in dict.fromkeys(keys):
        idx = np.array([l for l, k in enumerate(keys) if k == key])
        o = c_oracle.newton_solve(x0[idx], xr[idx[0]], ur[idx[0]], max_iters=max_iters, tol=tol, gamma_0=0.1,
                                  hist_len=max_iters)
        if out is None:
            out = {k: np.empty((len(x0),) + v.shape[1:], v.dtype) for k, v in o.items()}
        for k, v in o.items():
            out[k][idx] = v
    return out


def settle(eng, x0, xr, ur, idx, tol=1e-4, chunk=4096):
    """Both records of lanes ``idx`` of ``x0``; per lane: both sides' decisions, the first divergence (k, kind), the
    oracle's margin at k and its smallest margin before k, the largest cost difference before k, and for a "length"
    divergence the relative distance of max|sigma| from tol at the last iteration both ran (on both records).
    Per-lane references (xr (B,N,4), ur (B,T,2), B = len(x0)) follow their lanes.  Returns a dict of arrays."""
    idx = np.asarray(idx, np.int64)
    per_lane = np.ndim(xr) == 3
    keys = ("lane", "ng", "no", "sg", "so", "rg", "ro", "k", "kind", "margin_k", "margin_before", "smax_rel_o",
            "smax_rel_g", "pre_rel")
    out = {k: [] for k in keys}
    for lo in range(0, len(idx), chunk):
        sub = idx[lo:lo + chunk]
        xs, us = (xr[sub], ur[sub]) if per_lane else (xr, ur)
        ng, sg, rg, tg, hg, sm_g = gpu_record(eng, x0[sub], xs, us, tol)
        o = oracle_record(x0[sub], xs, us, tol)
        for j, lane in enumerate(sub):
            a, b = int(ng[j]), int(o["n_iter"][j])
            k, kind = first_divergence(tg[j], o["hist_trials"][j], hg[j], o["hist_cost"][j], a, b)
            m = o["hist_margin"][j]
            mk = float(m[k]) if k < b else np.inf
            mb = float(np.nanmin(m[:k])) if k > 0 else np.inf
            n = min(a, b)
            pre = np.abs(hg[j, :k] - o["hist_cost"][j, :k]) / np.maximum(np.abs(o["hist_cost"][j, :k]), 1e-300)
            pre = float(np.nanmax(pre)) if k > 0 and np.isfinite(pre).any() else 0.0
            so_rel = float(abs(o["hist_smax"][j, n - 1] - tol) / tol) if n > 0 else np.inf
            sg_rel = float(abs(sm_g[j, n - 1] - tol) / tol) if n > 0 else np.inf
            for key, v in zip(keys, (lane, a, b, sg[j], o["status"][j], rg[j], o["n_rollouts"][j], k, kind, mk, mb,
                                     so_rel, sg_rel, pre)):
                out[key].append(v)
    return {k: np.asarray(v) for k, v in out.items()}


def assert_settled(d, ng=None, sg=None, rg=None):
    """Every lane of a settle() record parts from the oracle at a tie of its own: the oracle's margin at the first
    divergent iteration below TIE ("trials" / "cost"), or max|sigma| within SMAX_TIE of tol ("length").  With the
    decisions of the run under test (ng, sg, rg), the record's re-run must reproduce them lane by lane."""
    if ng is not None:
        np.testing.assert_array_equal(d["ng"], ng)
        np.testing.assert_array_equal(d["sg"], sg)
        np.testing.assert_array_equal(d["rg"], rg)
    tie = d["kind"] != "length"
    bad = tie & ~(d["margin_k"] < TIE)
    assert not bad.any(), [(int(d["lane"][i]), int(d["k"][i]), str(d["kind"][i]), float(d["margin_k"][i]))
                           for i in np.nonzero(bad)[0][:10]]
    L = ~tie
    bad = L & ~((d["smax_rel_o"] < SMAX_TIE) | (d["smax_rel_g"] < SMAX_TIE))
    assert not bad.any(), [(int(d["lane"][i]), float(d["smax_rel_o"][i])) for i in np.nonzero(bad)[0][:10]]
