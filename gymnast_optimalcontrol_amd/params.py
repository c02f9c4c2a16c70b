"""Problem constants and parameter sets of the reference (host-side data only).

dynamics.py:15-61 (parameter sets), :173-175 (dt, ns, ni); trajectory_generation.py:8-18
(T, N, nu, nx, Q, R, Q_T).  The Newton/Armijo defaults are those of newton_Algorithm
(trajectory_generation.py:298, :345) and main.task_2 (main.py:65-71).
"""
DT = 2e-2
NS = 4
NI = 2
T_HORIZON = 10.0
N_KNOTS = int(T_HORIZON / DT) + 1   # 501

PARAM_NAMES = ("m1", "m2", "l1", "lc1", "l2", "lc2", "I1", "I2", "g", "f1", "f2")
PARAM_SETS = {
    1: dict(m1=1.0, m2=1.0, l1=1.0, lc1=1.0 / 2, l2=1.0, lc2=1.0 / 2, I1=0.33, I2=0.33, g=9.81, f1=1.0, f2=1.0),
    2: dict(m1=2.0, m2=2.0, l1=1.5, lc1=1.5 / 2, l2=1.5, lc2=1.5 / 2, I1=1.5, I2=1.5, g=9.81, f1=1.0, f2=1.0),
    3: dict(m1=1.5, m2=1.5, l1=2.0, lc1=2.0 / 2, l2=2.0, lc2=2.0 / 2, I1=2.0, I2=2.0, g=9.81, f1=1.0, f2=1.0),
}

Q_DIAG = (130.0, 30.0, 0.0001, 0.0001)
R_DIAG = (1e-6, 1.5)
QT_DIAG = (130.0, 130.0, 1.0, 1.0)

# newton_Algorithm defaults (trajectory_generation.py:298) and the line-search cap (:345)
NEWTON_DEFAULTS = dict(tol=1e-6, beta=0.7, c=0.5, gamma_0=1.0)
MAX_LINE_SEARCH_ITERS = 20
# main.task_2 (main.py:65-71)
TASK2 = dict(max_iters=5000, tol=1e-4, gamma_0=0.1)

import os as _os

# Task-2 problem input shipped with the package (a copy of the reference's
# trajectories_npz/fully_actuated_trajectory.npz, produced offline by fully_actuated_ref_gen.py).
DATA_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "data")
FULLY_ACTUATED_NPZ = _os.path.join(DATA_DIR, "fully_actuated_trajectory.npz")
