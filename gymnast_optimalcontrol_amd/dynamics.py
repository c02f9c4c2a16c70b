"""Drop-in for the reference's ``dynamics.py`` call surface, computed by the HIP engine.

Names, argument meaning and return conventions follow /root/reference/dynamics.py:
  dt, ns, ni (:173-175); dynamics(xx, uu) (:177-195, RK4); continuous_dynamics(xx, uu)
  (:197-213); Calculate_A_B_matrixes(x_t, u_t) -> (A_c, B_c) (:217-226); params_1/2/3 (:15-61);
  set_params(version_num) (:117-144), returning sympy matrices as the reference does; the symbolic layer
  (theta1, theta2, ..., M, C, Gvec, F, M_func, RHS_func, f_cont_sym, A_sym, B_sym, func_A, func_B, ...; :5-170)
  is built with sympy on first access (module __getattr__; ``from dynamics import *`` builds it, as importing
  the reference does).
Inputs are numpy arrays (as in the reference); the arithmetic runs in gfx950 kernels
(gym_rk4_step / gym_continuous_dynamics / gym_jacobians) and results come back as numpy.
Extensions: every function also accepts a stack of points (n,4)/(n,2) and returns (n,...);
``use_params(v)`` switches the parameter set the kernels integrate (in the reference the
dynamics are fixed to params_1 and set_params only feeds compute_equilibrium).
"""
from __future__ import annotations

import numpy as np

from .params import DT, NI, NS, PARAM_SETS

dt = DT
ns = NS
ni = NI

params_1 = dict(PARAM_SETS[1])
params_2 = dict(PARAM_SETS[2])
params_3 = dict(PARAM_SETS[3])

_engine = None
_pset = 1


def engine():
    """The process-wide HIP engine used by the reference-style functions (created lazily)."""
    global _engine
    if _engine is None:
        from .engine import AcrobotEngine
        _engine = AcrobotEngine(params=_pset, dt=dt)
    return _engine


def use_params(version_num: int = 1):
    """Switch the parameter set the kernels integrate (extension; see module docstring)."""
    global _engine, _pset
    if version_num not in PARAM_SETS:
        print("Invalid parameter version number, setting the default one.")
        version_num = 1
    _pset = version_num
    _engine = None
    return PARAM_SETS[version_num]


def set_params(version_num):
    """(M, C, G, F) of a parameter set as sympy matrices in theta1, theta2, theta1_dot, theta2_dot
    (dynamics.py:117-144), as the reference returns them (its compute_equilibrium lambdifies G over theta1,
    theta2); needs sympy.  set_params_numeric is the sympy-free numeric form."""
    from ._symbolic import set_params as sym
    return sym(version_num)


def set_params_numeric(version_num):
    """Numeric (M, C, G, F) of a parameter set (dynamics.py:117-144); no side effects.

    Returns callables M(th1, th2) (2,2), C(th1, th2, w1, w2) (2,2), G(th1, th2) (2,), and F (2,2),
    the numeric counterparts of the reference's substituted sympy matrices."""
    if version_num not in PARAM_SETS:
        print("Invalid parameter version number, setting the default one.")
        version_num = 1
    p = PARAM_SETS[version_num]
    m1, m2, l1, lc1, lc2, I1, I2, g = (p[k] for k in ("m1", "m2", "l1", "lc1", "lc2", "I1", "I2", "g"))

    def M(th1, th2):
        c2 = np.cos(th2)
        m12 = I2 + lc2 * m2 * (l1 * c2 + lc2)
        return np.array([[I1 + I2 + lc1**2 * m1 + m2 * (l1**2 + 2 * l1 * lc2 * c2 + lc2**2), m12],
                         [m12, I2 + lc2**2 * m2]])

    def Cm(th1, th2, w1, w2):
        h = l1 * lc2 * m2 * np.sin(th2)
        return np.array([[-h * w2, -h * (w1 + w2)], [h * w1, 0.0]])

    def G(th1, th2):
        s12 = np.sin(th1 + th2)
        return np.array([g * lc1 * m1 * np.sin(th1) + g * m2 * (l1 * np.sin(th1) + lc2 * s12), g * m2 * lc2 * s12])

    return M, Cm, G, np.diag([p["f1"], p["f2"]])


def _pts(xx, uu):
    x = np.asarray(xx, dtype=float)
    u = np.asarray(uu, dtype=float)
    single = x.squeeze().ndim == 1
    x = x.squeeze() if single else x
    u = u.squeeze() if single else u
    return x.reshape(-1, 4), u.reshape(-1, 2), single


def dynamics(xx, uu):
    """Discrete dynamics: one classic RK4 step of dt with uu held (dynamics.py:177-195)."""
    x, u, single = _pts(xx, uu)
    out = engine().rk4(x, u).cpu().numpy()
    return out[0] if single else out


def continuous_dynamics(xx, uu):
    """xdot = [qdot; M^-1 (tau - (C+F) qdot - G)], tau = [0, uu[1]] (dynamics.py:197-213)."""
    x, u, single = _pts(xx, uu)
    out = engine().continuous_dynamics(x, u).cpu().numpy()
    return out[0] if single else out


def Calculate_A_B_matrixes(x_t, u_t):
    """Continuous Jacobians (A_c (4,4), B_c (4,2)) at (x_t, u_t) (dynamics.py:217-226)."""
    x, u, single = _pts(x_t, u_t)
    A, B = engine().jacobians(x, u)
    A, B = A.cpu().numpy(), B.cpu().numpy()
    return (A[0], B[0]) if single else (A, B)


_SYMBOLIC = None


def __getattr__(name):
    """The reference's symbolic names (dynamics.py:5-170), built with sympy on first access."""
    global _SYMBOLIC
    from ._symbolic import NAMES
    if name not in NAMES:
        raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
    if _SYMBOLIC is None:
        from ._symbolic import model
        _SYMBOLIC = model()
    return _SYMBOLIC[name]


def _public():
    from ._symbolic import NAMES
    return ["dt", "ns", "ni", "params_1", "params_2", "params_3", "set_params", "dynamics", "continuous_dynamics",
            "Calculate_A_B_matrixes", *NAMES]


__all__ = _public()
