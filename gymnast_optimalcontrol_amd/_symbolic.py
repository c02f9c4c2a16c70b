"""The symbolic layer of the reference's ``dynamics.py`` (sympy), built on first use.

The reference builds its acrobot model symbolically at import time (/root/reference/dynamics.py:5-170): the
symbols, the matrices M, C, G, F of  M(q) q'' + (C(q, q') + F) q' + G(q) = tau,  their parameter-set-1
substitutions, the lambdified M_func / RHS_func, and the task-2 closed forms f_cont_sym, A_sym, B_sym with their
lambdified func_A, func_B, calc_continuous_dynamics.  The drop-in's numbers come from the HIP kernels, so none of
this is on the compute path; it exists so that reference callers that use the symbols (``from dynamics import *``;
``compute_equilibrium`` lambdifies ``set_params(1)[2]`` over ``theta1, theta2``, trajectory_generation.py:25-26)
run unchanged.  ``dynamics.__getattr__`` builds it lazily: importing the drop-in does not need sympy.
"""
from __future__ import annotations

from functools import lru_cache

from .params import PARAM_SETS

# the model's symbol names, in the reference's spelling (parameter-set dict keys are these strings; sympy's subs
# sympifies string keys, so the string-keyed params_1/2/3 substitute into these expressions)
PARAM_SYMBOLS = ("I1", "I2", "l1", "lc1", "l2", "lc2", "m1", "m2", "g", "f1", "f2")
STATE_SYMBOLS = ("theta1", "theta2", "theta1_dot", "theta2_dot")
INPUT_SYMBOLS = ("tau1", "tau2")


def _entries(sp, s):
    """The reference's module-level scalar entries M11 .. M22, C11 .. C22, G1, G2 (dynamics.py:64-83), unsimplified.
    They are mathematically equal to the reference's entries, not structurally: the factoring differs (e.g. G1 is
    g (m1 lc1 + m2 l1) sin(th1) + ..., M12 is d + h cos(th2)), so ``==`` / ``str()`` / ``.args`` comparisons against
    the reference's trees differ while ``simplify(a - b) == 0`` holds (tests/test_abi_host.py checks that).  M and
    Gvec simplify them entry by entry, as the reference does."""
    c2, s2 = sp.cos(s["theta2"]), sp.sin(s["theta2"])
    h = s["l1"] * s["lc2"] * s["m2"]                       # the coupling coefficient m2 l1 lc2
    d = s["I2"] + s["m2"] * s["lc2"] ** 2
    m_off = d + h * c2
    w1, w2 = s["theta1_dot"], s["theta2_dot"]
    s1, s12 = sp.sin(s["theta1"]), sp.sin(s["theta1"] + s["theta2"])
    g2 = s["g"] * s["m2"] * s["lc2"] * s12
    return {"M11": s["I1"] + s["m1"] * s["lc1"] ** 2 + s["m2"] * (s["l1"] ** 2 + s["lc2"] ** 2) + s["I2"] + 2 * h * c2,
            "M12": m_off, "M21": m_off, "M22": d,
            "C11": -h * s2 * w2, "C12": -h * s2 * (w1 + w2), "C21": h * s2 * w1, "C22": 0,
            "G1": s["g"] * (s["m1"] * s["lc1"] + s["m2"] * s["l1"]) * s1 + g2, "G2": g2}


def _mechanics(sp, s):
    """M, C, G, F of the double pendulum with joint friction (dynamics.py:63-90), from the symbol table s."""
    e = _entries(sp, s)
    Mm = sp.Matrix([[sp.simplify(e["M11"]), sp.simplify(e["M12"])], [sp.simplify(e["M21"]), sp.simplify(e["M22"])]])
    Cm = sp.Matrix([[e["C11"], e["C12"]], [e["C21"], e["C22"]]])
    Gv = sp.Matrix([[sp.simplify(e["G1"])], [sp.simplify(e["G2"])]])
    Fm = sp.diag(s["f1"], s["f2"])
    return Mm, Cm, Gv, Fm


@lru_cache(maxsize=None)
def model() -> dict:
    """Every public symbolic name of the reference's dynamics.py, keyed by that name."""
    import sympy as sp
    from sympy.utilities.lambdify import lambdify
    s = {n: sp.Symbol(n) for n in PARAM_SYMBOLS + STATE_SYMBOLS + INPUT_SYMBOLS}
    Mm, Cm, Gv, Fm = _mechanics(sp, s)
    out = dict(s)
    out.update(_entries(sp, s))
    out.update(M=Mm, C=Cm, Gvec=Gv, F=Fm)
    p1 = PARAM_SETS[1]
    out.update(M_num=Mm.subs(p1), C_num=Cm.subs(p1), G_num=Gv.subs(p1), F_num=Fm.subs(p1))
    q = [s["theta1"], s["theta2"]]
    qd = [s["theta1_dot"], s["theta2_dot"]]
    u = [s["tau1"], s["tau2"]]
    out.update(q_syms=q, qdot_syms=qd, all_syms=q + qd, u_syms=u, x_syms=q + qd,
               tau_vec=sp.Matrix(u), qdot_vec=sp.Matrix(qd))
    # fully actuated generic form (dynamics.py:108-115): q'' = M^-1 (tau - (C + F) q' - G), parameter set 1 in
    # C, G, F (M symbolic in its parameters, as the reference leaves it)
    rhs = sp.Matrix(u) - (out["C_num"] * sp.Matrix(qd) + out["F_num"] * sp.Matrix(qd) + out["G_num"])
    qdd = Mm.inv() * rhs
    f_gen = sp.Matrix(qd + list(qdd))
    out.update(RHS_expr=rhs, qddot_expr=qdd, f_expr=f_gen,
               M_func=lambdify(q, out["M_num"], "numpy"), RHS_func=lambdify(q + qd + u, rhs, "numpy"),
               A_expr=f_gen.jacobian(q + qd), B_expr=f_gen.jacobian(u))
    # task-2 acrobot (dynamics.py:146-170): tau = [0, tau2], parameter set 1 throughout
    Ms, Cs, Gs, Fs = set_params(1)
    x_vec = sp.Matrix(q + qd)
    u_vec = sp.Matrix(u)
    tau_a = sp.Matrix([0, s["tau2"]])
    rhs_a = tau_a - ((Cs + Fs) * sp.Matrix(qd) + Gs)
    qdd_a = Ms.LUsolve(rhs_a)
    f_cont = sp.Matrix.vstack(sp.Matrix(qd), qdd_a)
    A_s, B_s = f_cont.jacobian(x_vec), f_cont.jacobian(u_vec)
    args = list(x_vec) + list(u_vec)
    out.update(M_sym=Ms, C_sym=Cs, G_sym=Gs, F_sym=Fs, q_vec=sp.Matrix(q), x_vec=x_vec, u_vec=u_vec,
               tau_acrobot=tau_a, RHS_sym=rhs_a, qddot_sym=qdd_a, f_cont_sym=f_cont, A_sym=A_s, B_sym=B_s,
               calc_continuous_dynamics=lambdify(args, f_cont, "numpy"), func_A=lambdify(args, A_s, "numpy"),
               func_B=lambdify(args, B_s, "numpy"))
    return out


def set_params(version_num):
    """(M, C, G, F) as sympy matrices with parameter set ``version_num`` substituted (dynamics.py:117-144); an
    unknown number prints the reference's message and uses set 1."""
    import sympy as sp
    if version_num not in PARAM_SETS:
        print("Invalid parameter version number, setting the default one.")
        version_num = 1
    s = {n: sp.Symbol(n) for n in PARAM_SYMBOLS + STATE_SYMBOLS + INPUT_SYMBOLS}
    p = PARAM_SETS[version_num]
    return tuple(m.subs(p) for m in _mechanics(sp, s))


NAMES = (PARAM_SYMBOLS + STATE_SYMBOLS + INPUT_SYMBOLS +
         ("M11", "M12", "M21", "M22", "C11", "C12", "C21", "C22", "G1", "G2") +
         ("M", "C", "Gvec", "F", "M_num", "C_num", "G_num", "F_num", "q_syms", "qdot_syms", "all_syms", "u_syms",
          "x_syms", "tau_vec", "qdot_vec", "RHS_expr", "qddot_expr", "f_expr", "M_func", "RHS_func", "A_expr",
          "B_expr", "M_sym", "C_sym", "G_sym", "F_sym", "q_vec", "x_vec", "u_vec", "tau_acrobot", "RHS_sym",
          "qddot_sym", "f_cont_sym", "A_sym", "B_sym", "calc_continuous_dynamics", "func_A", "func_B"))
