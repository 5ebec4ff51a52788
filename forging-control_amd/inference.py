"""Batched closed-loop inference on the rollout kernel.

The reference's closed-loop harness steps, per trajectory and per sampling instant, the LSTM surrogate
on a 10-row window (``NeuralNetwork.simulator_make_step``, Functions.py:969-1011, window built at
:1196-1207) and the FNN controller (``FeasibilityRecovery.NN_make_step``, :1560-1613, without the
CasADi feasibility recovery). Here the LSTM step is one window of the fused gfx950 forward
(``fcr_forward`` with N = 1 and u0 = the window's last command, no backward state) over a whole batch
of trajectories; the controller is the 3->50->1 FNN.
"""
from __future__ import annotations

import numpy as np
import torch

from .functions import _simulator_params
from .rollout import WINDOW_ROWS, rollout


def simulate_step(simulator, windows: torch.Tensor, noise: torch.Tensor | None = None) -> torch.Tensor:
    """x̂ = LSTMModel(window) (+ noise) for every window of a (B, 10, 5) batch on a ROCm device: the
    scaled prediction of ``simulator_make_step`` before ``scalers['output'].inverse_transform``."""
    if windows.dim() != 3 or windows.shape[1:] != (WINDOW_ROWS, 5):
        raise ValueError(f"windows must be (B, 10, 5), got {tuple(windows.shape)}")
    B, dev = windows.shape[0], windows.device
    f32 = dict(dtype=torch.float32, device=dev)
    zero_ctrl = (torch.zeros(1, 3, **f32), torch.zeros(1, **f32), torch.zeros(1, 1, **f32))   # unused at N = 1
    with torch.no_grad():
        w = windows.to(torch.float32).contiguous()
        out = rollout(torch.zeros(B, 3, **f32), w[:, WINDOW_ROWS - 1, 4].contiguous(), w, zero_ctrl,
                      tuple(_to(p, dev) for p in _flat(_simulator_params(simulator))), 1, 0.0,
                      None if noise is None else noise.to(**f32).reshape(B, 1, 4))
    return out[5][:, 0, :]


def controller_step(controller, X: torch.Tensor) -> torch.Tensor:
    """u = FNNModel(X) for a (B, 3) batch of scaled controller inputs (the NN part of NN_make_step)."""
    with torch.no_grad():
        return controller(X)


def simulator_make_step(X: np.ndarray, model, scalers: dict, noise: np.ndarray, device=None) -> np.ndarray:
    """Drop-in for ``NeuralNetwork.simulator_make_step`` (Functions.py:969-1011) with the same arguments:
    X (B, 10, 5) or (10, 5) scaled LSTM inputs, noise (4,) or (B, 4) in scaled units; returns the unscaled
    prediction ``scalers['output'].inverse_transform(model(X) + noise)``.

    ``device`` defaults to where the model's weights are. A model on a ROCm device runs the whole batch
    through the fused gfx950 forward; a model the harness moved to the CPU (UL/Main.py:347-348) runs
    ``model(X_new, "cpu")`` exactly as the reference does — its own ``nn.LSTM`` (LSTMModel.forward)."""
    if device is None:
        device = next(model.parameters()).device
    device = torch.device(device)
    Xt = torch.as_tensor(np.asarray(X, np.float32), device=device)
    if Xt.dim() == 2:
        Xt = Xt.unsqueeze(0)
    nz = torch.as_tensor(np.broadcast_to(np.asarray(noise, np.float32), (Xt.shape[0], 4)).copy(), device=device)
    if device.type == "cpu":
        model.eval()
        with torch.no_grad():
            y = (model(Xt, "cpu") + nz).numpy()
        return scalers["output"].inverse_transform(y)
    y = simulate_step(model, Xt, nz).cpu().numpy().astype(np.float64)
    return scalers["output"].inverse_transform(y)


def _flat(params):
    w_ih, w_hh, fc_w, fc_b = params
    return (list(w_ih), list(w_hh), fc_w, fc_b)


def _to(p, dev):
    if isinstance(p, list):
        return [t.detach().to(dev) for t in p]
    return p.detach().to(dev)
