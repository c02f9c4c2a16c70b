"""Report surface of the drop-in trajectory_generation (CPU: plotting only, no kernel launch).

main.task_2 calls tg.generate_report_graphs (main.py:82; trajectory_generation.py:405-509) after the solve, and
main.task_1 calls tg.plot_results (main.py:49, absent from the reference module)."""
import numpy as np

from conftest import load_golden


def test_report_iterations_selection():
    from gymnast_optimalcontrol_amd.trajectory_generation import report_iterations
    assert report_iterations(394) == [0, 1, 5, 10, 98, 100, 196, 294, 393]
    assert report_iterations(3) == [0, 1, 2]
    assert report_iterations(1) == [0]


def test_generate_report_graphs_from_task2_history():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    from gymnast_optimalcontrol_amd import trajectory_generation as tg
    g = load_golden("task2_solve")
    n = len(g["cost_hist"])
    # history as newton_Algorithm fills it (the fixture keeps 4 of the 394 trajectories: repeat them)
    x_trajs = [g["x_hist"][min(np.searchsorted(g["x_hist_idx"], i), 3)] for i in range(n)]
    hist = {"cost": list(g["cost_hist"]), "sigma_norm": list(g["sigma_norm_hist"]), "x_trajs": x_trajs,
            "sigmas": [list(g["sigma_first"])] + [list(g["sigma"])] * (n - 2)}
    u_full = np.vstack([g["u_ref"], g["u_ref"][-1:]])               # u_ref with N rows is trimmed (:407-410)
    d = tg.generate_report_graphs(g["t_ref"], g["x_ref"], u_full, g["x"], g["u"], hist)
    assert d["iterations_shown"] == [0, 1, 5, 10, 98, 100, 196, 294, 393]
    assert d["sigma_iterations"] == [0, 1, 2, n - 2]
    np.testing.assert_array_equal(d["sigma_tau2"][0], g["sigma_first"][:, 1])
    assert len(d["figures"]) == 4
    assert tg.plot_results is tg.generate_report_graphs
    plt.close("all")
