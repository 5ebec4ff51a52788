"""fp64 PyTorch restatement of one LSTM-surrogate training step (TEST INFRASTRUCTURE ONLY).

Restates NeuralNetwork.train_model's body (Model_NN/Functions.py:541-566) for LSTMModel(5, H, 4, 3)
(Model_NN/Functions.py:255-330: nn.LSTM without bias from a zero state, fc on the last step) with
nn.MSELoss (Model_NN/Main.py:229) — forward, loss, and autograd's gradient of every weight and of the
input — in float64 on the CPU with stock torch operators (the reference's arithmetic lives in torch).

PARITY STATUS: unpinned by reference fixtures (the reference ships none for this path and its Python
may not be run here); autograd is cross-checked by central finite differences in
tests/test_surrogate.py.
"""
from __future__ import annotations

import torch

from .rollout_torch import TorchLSTM


def build(params, dtype=torch.float64):
    H = params["Whh"][0].shape[1]
    m = TorchLSTM(5, H, 4, 3).to(dtype)
    with torch.no_grad():
        for k in range(3):
            getattr(m.lstm, f"weight_ih_l{k}").copy_(torch.as_tensor(params["Wih"][k], dtype=dtype))
            getattr(m.lstm, f"weight_hh_l{k}").copy_(torch.as_tensor(params["Whh"][k], dtype=dtype))
        m.fc.weight.copy_(torch.as_tensor(params["fcW"], dtype=dtype))
        m.fc.bias.copy_(torch.as_tensor(params["fcb"], dtype=dtype))
    return m


def step_grads(params, x, target, dtype=torch.float64):
    """(y, loss, grads) with grads = {'Wih': [3], 'Whh': [3], 'fcW', 'fcb', 'x'} as numpy float64."""
    m = build(params, dtype)
    xt = torch.as_tensor(x, dtype=dtype).clone().requires_grad_(True)
    y = m(xt)
    loss = torch.nn.functional.mse_loss(y, torch.as_tensor(target, dtype=dtype))
    loss.backward()
    g = {"Wih": [getattr(m.lstm, f"weight_ih_l{k}").grad.numpy() for k in range(3)],
         "Whh": [getattr(m.lstm, f"weight_hh_l{k}").grad.numpy() for k in range(3)],
         "fcW": m.fc.weight.grad.numpy(), "fcb": m.fc.bias.grad.numpy(), "x": xt.grad.numpy()}
    return y.detach().numpy(), float(loss), g


def train_steps(params, batches, lr=1e-3, weight_decay=0.0, dtype=torch.float64):
    """AdamW (Model_NN/Main.py:232: lr, weight_decay=0.0) over (x, target) batches; returns the final
    parameters as numpy float64 and the per-step losses."""
    m = build(params, dtype)
    opt = torch.optim.AdamW(m.parameters(), lr=lr, weight_decay=weight_decay)
    losses = []
    for x, target in batches:
        opt.zero_grad()
        loss = torch.nn.functional.mse_loss(m(torch.as_tensor(x, dtype=dtype)), torch.as_tensor(target, dtype=dtype))
        loss.backward()
        opt.step()
        losses.append(float(loss))
    out = {"Wih": [getattr(m.lstm, f"weight_ih_l{k}").detach().numpy() for k in range(3)],
           "Whh": [getattr(m.lstm, f"weight_hh_l{k}").detach().numpy() for k in range(3)],
           "fcW": m.fc.weight.detach().numpy(), "fcb": m.fc.bias.detach().numpy()}
    return out, losses
