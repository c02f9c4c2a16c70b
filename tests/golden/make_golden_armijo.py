"""Golden fixture for the Armijo line-search report (plot_armijo_line_search, trajectory_generation.py:254-296).

Test infrastructure only; runs in the build container against the read-only reference (recipe of
make_golden.py / SURVEY.md 8(c)).  The reference's plot_armijo_line_search computes its 200-point
curve J(gamma) (:256-264) and hands it to matplotlib; this script runs main.task_2's solve
(main.py:65-71) for 7 iterations with plot_armijo_iters=7, replaces the module's ``plt`` with a
recorder, and stores what the reference plotted -- the curve (steps, costs), the first-order model and
the Armijo line (:268-279), the tested step sizes and costs and the accepted step (:282-287) -- for the
plotted iterations 0, 1, 2, 4, 6, plus the full inputs (x, u, K, sigma, J, dJ) of iteration 0.

Usage:  python tests/golden/make_golden_armijo.py
"""
import contextlib
import io
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, _import_reference  # noqa: E402


class _Recorder:
    """Stands in for matplotlib.pyplot: keeps plot/scatter arguments, ignores everything else."""

    def __init__(self):
        self.calls = []

    def plot(self, *a, **k):
        self.calls.append(("plot", [np.asarray(v, dtype=float) for v in a]))

    def scatter(self, *a, **k):
        self.calls.append(("scatter", [np.asarray(v, dtype=float) for v in a]))

    def __getattr__(self, name):
        return lambda *a, **k: None


def main():
    tg = _import_reference()   # its plot_armijo_line_search is stubbed: reload the module for the real one
    import importlib
    fresh = importlib.reload(tg)
    rec = _Recorder()
    fresh.plt = rec
    real = fresh.plot_armijo_line_search
    seen = []

    def wrapped(iteration, x_traj, u_traj, K, sigma, cost_current, x_ref, u_ref, delta_J, gamma_accepted,
                stepsizes_tested, costs_tested, c=0.5, beta=0.7):
        n0 = len(rec.calls)
        real(iteration, x_traj, u_traj, K, sigma, cost_current, x_ref, u_ref, delta_J, gamma_accepted,
             stepsizes_tested, costs_tested, c, beta)
        calls = rec.calls[n0:]
        seen.append(dict(k=iteration, x=np.array(x_traj), u=np.array(u_traj), K=np.array(K), sigma=np.array(sigma),
                         J=float(cost_current), dJ=float(delta_J), gamma=float(gamma_accepted),
                         tested=np.array(stepsizes_tested, dtype=float), costs_tested=np.array(costs_tested),
                         steps=calls[0][1][0], costs=calls[0][1][1], lin=calls[1][1][1], arm=calls[2][1][1]))

    fresh.plot_armijo_line_search = wrapped
    x_ref, u_ref, _ = fresh.get_fully_actuated_ref()
    with contextlib.redirect_stdout(io.StringIO()):
        fresh.newton_Algorithm(np.zeros(4), x_ref, u_ref, max_iters=7, tol=1e-4, gamma_0=0.1, plot_armijo_iters=7)
    ks = [d["k"] for d in seen]
    assert ks == [0, 1, 2, 4, 6], ks
    out = {"iters": np.array(ks), "x_ref": x_ref, "u_ref": u_ref}
    for d in seen:
        p = f"k{d['k']}_"
        for key in ("steps", "costs", "lin", "arm", "tested", "costs_tested"):
            out[p + key] = d[key]
        for key in ("J", "dJ", "gamma"):
            out[p + key] = np.float64(d[key])
    d0 = seen[0]
    for key in ("x", "u", "K", "sigma"):
        out["k0_" + key] = d0[key]
    np.savez_compressed(os.path.join(OUT, "armijo_sweep.npz"), **out)
    print("wrote armijo_sweep.npz", {k: v.shape for k, v in out.items() if k.startswith("k0_")})


if __name__ == "__main__":
    main()
