"""Batched closed-loop evaluation on the GPU (SURVEY.md §8(f) ranks 1 + 2 together).

The reference evaluates its trained controller in ``NeuralNetwork.loop`` (Functions.py:1075-1240): for
each trajectory and step, the speed reference from ``tvp_fun`` (:926-966), the controller through
``FeasibilityRecovery.NN_make_step`` (:1560-1613, MaxAbs-scaled inputs, fp32 torch model, unscaled
output) and the press advanced by do-mpc's simulator — one trajectory at a time, in Python.
:class:`ClosedLoop` runs the controller and the press (the reference's RK4 integrator ``F`` of
``Ruge_Kuta``, Functions.py:1743-1781, on ``forging_model`` or the smooth ``template_model``) for a whole
batch of trajectories and all steps in ONE kernel launch (``fcr_closed_loop_run``,
forging-control_amd/csrc/fcr_closed_loop.h). Feasibility recovery (CasADi/IPOPT) and do-mpc's process
and measurement noise are not part of it.
"""
from __future__ import annotations

import ctypes
import random

import numpy as np
import torch

from . import _native
from .functions import _controller_params
from .plant import SUBSTEPS_REFERENCE, TS_REFERENCE


def tvp_fun(t_now: float, ref_step: float, bias_work: int, bias_return: int, epsilon: float = 1e-7) -> float:
    """NeuralNetwork.tvp_fun (Functions.py:926-966): a random working-stroke speed in [0.1, 0.9] for the
    first half of every reference period and a random return-stroke speed in [-0.9, -0.1] for the second,
    each drawn from Python's generator seeded by the period index plus a bias."""
    phase = (t_now + epsilon) % ref_step
    period = (t_now + epsilon) // ref_step
    if phase < ref_step / 2:
        random.seed(period + bias_work)
        return 0.8 * random.random() + 0.1
    random.seed(period + bias_return)
    return -0.8 * random.random() - 0.1


def reference_speeds(n_traj: int, t_traj: int, ts: float, bias_work: int, bias_return: int) -> np.ndarray:
    """(n_traj, t_traj) references the harness uses: t_now = (idx·T_traj + t)·Ts, period Ts·T_traj
    (Functions.py:1116-1160)."""
    t_ref = ts * t_traj
    return np.array([[tvp_fun((i * t_traj + t) * ts, t_ref, bias_work, bias_return) for t in range(t_traj)]
                     for i in range(n_traj)])


def _scale(s):
    """A MaxAbsScaler's ``scale_`` (sklearn object or plain number/array)."""
    return np.atleast_1d(np.asarray(getattr(s, "scale_", s), dtype=np.float64))


class ClosedLoop:
    """Controller + press for B trajectories over T steps: ``run(x0 (B,5), ref (B,T))`` ->
    ``(x (B,T+1,5), u (B,T))`` as fp64 device tensors.

    ``scalers`` holds the controller's MaxAbs scalers as NN_make_step reads them: ``'input'`` (scale_ of
    [y_dot, z, ref]; the first two are used), ``'y_dot'`` (scales the reference) and ``'output'``."""

    def __init__(self, controller, scalers: dict, ts: float = TS_REFERENCE, substeps: int = SUBSTEPS_REFERENCE,
                 smooth: bool = True):
        self.controller = controller
        s_in = _scale(scalers["input"])
        self.in_scale = (float(s_in[0]), float(s_in[1]))
        self.ref_scale = float(_scale(scalers["y_dot"])[0])
        self.out_scale = float(_scale(scalers["output"])[0])
        self.ts, self.substeps, self.smooth = float(ts), int(substeps), bool(smooth)

    def run(self, x0: torch.Tensor, ref: torch.Tensor):
        dev = x0.device
        if dev.type != "cuda" or ref.device != dev:
            raise RuntimeError(f"ClosedLoop runs on a ROCm device only (x0 on {x0.device}, ref on {ref.device})")
        if x0.dim() != 2 or x0.shape[1] != 5 or ref.dim() != 2 or ref.shape[0] != x0.shape[0]:
            raise ValueError(f"x0 must be (B,5) and ref (B,T); got {tuple(x0.shape)}, {tuple(ref.shape)}")
        B, T = x0.shape[0], ref.shape[1]
        W_inp, b_inp, W_out = (p.detach().to(device=dev, dtype=torch.float32).contiguous()
                               for p in _controller_params(self.controller))
        x0c = x0.to(torch.float64).contiguous()
        refc = ref.to(torch.float64).contiguous()
        x = torch.empty(B, T + 1, 5, dtype=torch.float64, device=dev)
        u = torch.empty(B, T, dtype=torch.float64, device=dev)
        p = lambda t: t.data_ptr()
        args = _native.FcrClosedLoop(B, T, self.ts, self.substeps, int(self.smooth), p(x0c), p(refc), p(W_inp),
                                     p(b_inp), p(W_out), W_inp.shape[0], (ctypes.c_double * 2)(*self.in_scale),
                                     self.ref_scale, self.out_scale, p(x), p(u))
        _native.check(_native.load().fcr_closed_loop_run(ctypes.byref(args),
                                                         ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
                      "fcr_closed_loop_run")
        return x, u
