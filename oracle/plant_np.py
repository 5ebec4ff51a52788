"""fp64 NumPy restatement of the open-die forging plant and its RK4 integrator.

TEST INFRASTRUCTURE ONLY. Nothing in the product package imports this module; only ``tests/`` and the
plant benchmark's CPU-baseline leg use it, and only as the checker.

What it restates (paths relative to ``/root/reference/Unsupervised Learning/``):

* ``FeasibilityRecovery.forging_model``  Functions.py:1615-1740 -> :func:`forging_rhs` (``smooth=False``)
  — the press dynamics as CasADi builds them for the feasibility-recovery integrator;
* ``template_model``                     template_model.py:19-149 -> :func:`forging_rhs` (``smooth=True``)
  — the same dynamics with pressures floored by the C^1 ``smooth_relu`` (:106-118), the model do-mpc
  simulates;
* ``FeasibilityRecovery.Ruge_Kuta``      Functions.py:1743-1781 -> :func:`rk4_step`
  — M = 4 classical RK4 sub-steps of TS/M, command held over the step;
* the harness's state update ``x_{t+1} = F(x_t, u_t)`` over a trajectory -> :func:`trajectory`.

CasADi semantics kept: ``if_else(c, a, b)`` evaluates both branches and masks the untaken one to 0
(``if_else_zero``), so NaN/inf in the untaken ``Fd_article`` branch never leaks; ``sign(0) = 0``.
All arithmetic is fp64 like CasADi's SX evaluation.

PARITY STATUS: pinned coarsely (not to rounding): the reference ships closed-loop traces
(``results/MPC_dataframe.txt``, ``results/Unsupervised_dataframe.txt``, ``%.6f``; the harness writes
them from do-mpc's CVODES simulator, possibly with process noise) and ``tests/golden/plant_trace.npz``
holds their rows as data; ``tests/test_plant.py`` checks that one RK4 step of this restatement from row
t with command u_t lands on row t+1 to a median relative error below 2e-4 per state (observed ~5e-5).
"""
from __future__ import annotations

import numpy as np

# Press / oil / material constants, Functions.py:1636-1700 (= template_model.py:19-92)
M_MASS = 90000.0
B_DAMP = 25000.0
FT = 200000.0
D1, D2 = 0.6, 0.5
A1 = np.pi * D1 ** 2 / 4
A2 = np.pi * D2 ** 2 / 4
G = 9.81
KB = 22 * 10 ** 9
V1_0, V2_0 = 0.3, 0.1
KL_1, KL_2 = 8 * 10 ** (-13), 14 * 10 ** (-14)
CD, RHO, D = 0.63, 858.0, 0.006
PS, PT = 32 * 10 ** 6, 101325.0
MU, K, W0, H0, B0 = 0.3, 1.115, 0.2, 0.5, 0.1
A_SPREAD = 0.14 + 0.36 * (B0 / W0) - 0.054 * (B0 / W0) ** 2
T_DEF = 900.0
T1 = 0.005
M0, M1, M2, M3, M4 = 1200 * 10 ** 6, -0.0025, -0.0587, 0.1165, -0.0065
SMOOTH_EPS = 1e-6          # template_model.py:113


def _smooth_relu(x):
    return 0.5 * (x + np.sqrt(x * x + SMOOTH_EPS))


def forging_rhs(x: np.ndarray, u: np.ndarray, smooth: bool = False) -> np.ndarray:
    """xdot for states x (..., 5) = [y, y_dot, p1, p2, z] and command u (...), Functions.py:1633-1740."""
    x = np.asarray(x, np.float64)
    u = np.asarray(u, np.float64)
    y, yd, p1, p2, z = (x[..., k] for k in range(5))
    if smooth:                                   # template_model.py:116-117 (P_MIN = 0)
        p1 = _smooth_relu(p1)
        p2 = _smooth_relu(p2)
    h1 = H0 - y
    with np.errstate(all="ignore"):
        w1 = W0 * (H0 / h1) ** A_SPREAD
        b1 = B0 * (1 + 0.67 * (H0 / h1 * W0 / w1 - 1))
        kd = K * (1 + MU * b1 / (2 * y) + y / (4 * b1))
        ad = w1 * b1
        e = np.log(H0 / (H0 - y))
        e_dot = yd / (H0 - y)
        fd = kd * ad * M0 * np.exp(M1 * T_DEF) * e ** M2 * e_dot ** M3 * np.exp(M4 / e)
    fd = np.where((y > 0) & (yd >= 0), fd, 0.0)   # if_else(logic_and(y>0, y_dot>=0), ..., 0)

    def q(a):
        return np.pi * D * z * CD * np.sqrt(2 / RHO * np.abs(a)) * np.sign(a)

    qv_pb = np.where(z >= 0, q(PS - p1), q(p1 - PT))
    qv_at = np.where(z >= 0, q(p2 - PT), q(PS - p2))
    v1 = V1_0 / 2 + A1 * y
    v2 = V2_0 / 2 - A2 * y
    ft = np.where(np.abs(yd) <= 0.5, FT * yd / 0.5, FT)
    return np.stack([
        yd,
        (3 * np.pi * D1 ** 2 * p1 / 4 - np.pi * D2 ** 2 * p2 / 2 - B_DAMP * yd - ft - fd) / M_MASS + G,
        KB / v1 * (qv_pb / 3 - A1 * yd - KL_1 * p1),
        KB / v2 * (-qv_at / 2 + A2 * yd - KL_2 * p2),
        -z / T1 + u / T1,
    ], axis=-1)


def rk4_step(x, u, ts: float = 1e-3, substeps: int = 4, smooth: bool = False) -> np.ndarray:
    """F(x0, u) of Functions.py:1758-1779: `substeps` RK4 steps of ts/substeps, u held."""
    dt = ts / substeps
    x = np.asarray(x, np.float64)
    for _ in range(substeps):
        k1 = forging_rhs(x, u, smooth)
        k2 = forging_rhs(x + dt / 2 * k1, u, smooth)
        k3 = forging_rhs(x + dt / 2 * k2, u, smooth)
        k4 = forging_rhs(x + dt * k3, u, smooth)
        x = x + dt / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
    return x


def trajectory(x0, U, ts: float = 1e-3, substeps: int = 4, smooth: bool = False) -> np.ndarray:
    """x (B, S+1, 5): x[:, 0] = x0 (B, 5), x[:, t+1] = F(x[:, t], U[:, t]) for U (B, S)."""
    x0 = np.asarray(x0, np.float64)
    U = np.asarray(U, np.float64)
    out = np.empty((x0.shape[0], U.shape[1] + 1, 5))
    out[:, 0] = x0
    x = x0
    for t in range(U.shape[1]):
        x = rk4_step(x, U[:, t], ts, substeps, smooth)
        out[:, t + 1] = x
    return out
