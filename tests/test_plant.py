"""Batched forging-press plant: oracle pinned on the reference's traces (CPU),
the C ABI's argument checks (CPU), and the fp64 HIP integrator against the oracle (GPU)."""
import importlib
import os

import numpy as np
import pytest
import torch

from oracle.plant_np import forging_rhs, rk4_step, trajectory
from tests.conftest import GOLDEN

fca = importlib.import_module("forging-control_amd")

TRACE = os.path.join(GOLDEN, "plant_trace.npz")
PS_EQ = 32e6          # supply pressure, Functions.py:1660: the working flow's sign(PS - p1) is 0 there


def _trace_transitions(name):
    d = np.load(TRACE)[name]
    # row t+1 holds the state the command u_{t+1} (logged on that row) produced from row t
    return d[:-1, 2:7], d[1:, 7], d[1:, 2:7], np.abs(d[:, 2:7]).max(0)


@pytest.mark.parametrize("name", ["mpc", "unsupervised"])
@pytest.mark.parametrize("smooth", [False, True])
def test_oracle_reproduces_reference_traces(name, smooth):
    """One RK4 step (TS = 1 ms, M = 4, Functions.py:1743-1781) of the restated dynamics from each logged
    state lands on the next logged state. The traces come from do-mpc's CVODES run of the reference
    plant and are printed %.6f, so this pins the equations and constants, not the rounding: per state
    the median error is ~1e-6 of the state's range (a 1 % change of any constant moves it >10x)."""
    x, u, x_next, scale = _trace_transitions(name)
    rel = np.abs(rk4_step(x, u, 1e-3, 4, smooth) - x_next) / scale
    assert np.all(np.median(rel, axis=0) < 1e-5), np.median(rel, axis=0)
    # a handful of transitions at the reference switches do not follow the logged command
    assert np.mean(rel.max(axis=1) < 1e-4) > 0.95


def test_oracle_casadi_if_else_semantics():
    """Fd_article is masked to 0 off its branch even where its formula is NaN (y <= 0, log of <= 0),
    and sign(0) = 0 in the valve flows (Functions.py:1704, :1709-1715)."""
    x = np.array([[0.0, 0.3, 1e7, 5e6, 0.1], [-0.01, -0.2, 1e7, 5e6, -0.1], [0.05, 0.0, PS_EQ, 5e6, 0.1]])
    f = forging_rhs(x, np.array([0.1, 0.1, 0.1]))
    assert np.all(np.isfinite(f))
    # y = 0 -> no deformation force: y_dot only sees damping B and friction FT·y_dot/0.5 (:1726)
    f_still = forging_rhs(x[:1] * [1, 0, 1, 1, 1], 0.1)[0, 1]
    assert f[0, 1] == pytest.approx(f_still - (25000 * 0.3 + 200000 * 0.3 / 0.5) / 90000)
    assert np.all(np.isfinite(trajectory(x, np.full((3, 20), 0.2))))


def test_host_refuses_cpu_tensors():
    with pytest.raises(RuntimeError, match="ROCm device only"):
        fca.forging_rk4(torch.zeros(4, 5, dtype=torch.float64), torch.zeros(4, 3, dtype=torch.float64))


@pytest.mark.parametrize("args,msg", [
    ((-1, 3, 1e-3, 4, 0), "B="), ((4, -2, 1e-3, 4, 0), "S="), ((4, 3, 0.0, 4, 0), "ts="),
    ((4, 3, 1e-3, 0, 0), "substeps="), ((4, 3, 1e-3, 4, 2), "smooth="), ((4, 3, 1e-3, 4, 0), "NULL"),
])
def test_abi_rejects_bad_arguments_before_any_device_call(args, msg):
    lib = fca._native.load()
    rc = lib.fcr_plant_rk4(*args, None, None, None, None)
    assert rc == -1 and msg in lib.fcr_last_error().decode()


def test_abi_empty_batch_is_a_noop():
    assert fca._native.load().fcr_plant_rk4(0, 5, 1e-3, 4, 0, None, None, None, None) == 0


# ------------------------------------------------------------------------------------------------ GPU

def _realistic_batch(B, S, seed):
    """States and commands spread around the reference's closed-loop traces (work and return strokes)."""
    rng = np.random.default_rng(seed)
    d = np.concatenate([np.load(TRACE)["mpc"], np.load(TRACE)["unsupervised"]])
    rows = d[rng.integers(0, len(d), B)]
    x0 = rows[:, 2:7] * (1 + 0.05 * rng.standard_normal((B, 5)))
    u = rows[:, 7:8] + 0.05 * np.cumsum(rng.standard_normal((B, S)), axis=1) / np.sqrt(S)
    return x0, u


def _max_rel(a, b):
    scale = np.abs(b).reshape(-1, 5).max(0)
    return (np.abs(a - b).reshape(-1, 5) / scale).max(0)


@pytest.mark.gpu
@pytest.mark.parametrize("smooth", [False, True])
@pytest.mark.parametrize("B,S,substeps", [(1, 1, 4), (333, 25, 4), (2048, 40, 4), (64, 10, 1), (130, 7, 9)])
def test_gpu_plant_matches_oracle(smooth, B, S, substeps):
    x0, u = _realistic_batch(B, S, seed=B + S)
    ref = trajectory(x0, u, 1e-3, substeps, smooth)
    dev = torch.device("cuda:0")
    got = fca.forging_rk4(torch.tensor(x0, device=dev), torch.tensor(u, device=dev), 1e-3, substeps, smooth)
    got = got.cpu().numpy()
    assert got.shape == (B, S + 1, 5)
    assert np.array_equal(got[:, 0], x0)
    err = _max_rel(got, ref)
    assert np.all(err < 1e-9), err


@pytest.mark.gpu
def test_gpu_plant_open_loop_on_reference_commands():
    """The MPC trace's 600 commands from its first state, open loop, kernel vs oracle over every step."""
    d = np.load(TRACE)["mpc"]
    x0, u = d[:1, 2:7], d[1:, 7][None, :]
    for smooth in (False, True):
        ref = trajectory(x0, u, 1e-3, 4, smooth)
        got = fca.ForgingRK4(1e-3, 4, smooth).rollout(torch.tensor(x0, device="cuda:0"),
                                                       torch.tensor(u, device="cuda:0")).cpu().numpy()
        assert np.all(_max_rel(got, ref) < 1e-9)


@pytest.mark.gpu
def test_gpu_plant_single_step_call_convention():
    """F(x0=..., u=...)['xf'] of the batched integrator = one oracle RK4 step per trajectory."""
    x0, u = _realistic_batch(97, 1, seed=5)
    F = fca.ForgingRK4()
    xf = F(torch.tensor(x0, device="cuda:0"), torch.tensor(u[:, 0], device="cuda:0"))["xf"].cpu().numpy()
    assert np.all(_max_rel(xf, rk4_step(x0, u[:, 0])) < 1e-12)
