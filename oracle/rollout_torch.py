"""PyTorch-CPU restatement of the MPC rollout loss, in the reference's op order.

TEST INFRASTRUCTURE ONLY (checker and CPU baseline). The product package never imports it.

PARITY STATUS: *parity unpinned* — see ``oracle/rollout_np.py``'s header and DESIGN.md §Oracle. This
module is the second, independent restatement the NumPy oracle is cross-checked against: it runs the
same stock ``torch`` operators the reference runs (``nn.LSTM`` without bias, ``nn.Linear``, ReLU,
Hardtanh, autograd), in the order of ``MPCLoss.forward``
(``/root/reference/Unsupervised Learning/Functions.py:1386-1472``). Because the reference's arithmetic
lives in torch itself, this is also the "reference CPU path" timed by ``bench.py``'s
``cpu_baseline`` leg (kind ``"port"``): it keeps the reference's ``requires_grad`` on the frozen LSTM
weights, so torch also spends the (unused) LSTM weight-gradient work the reference spends.
"""
from __future__ import annotations

import torch
from torch import nn

P1_MAX = 2.122366
P2_MAX = 1.036233


class TorchLSTM(nn.Module):
    """Stacked LSTM surrogate with a linear readout (Functions.py:317-379)."""

    def __init__(self, in_dim=5, hidden=50, out_dim=4, layers=3):
        super().__init__()
        self.hidden, self.layers = hidden, layers
        self.lstm = nn.LSTM(in_dim, hidden, layers, batch_first=True, bias=False)
        self.fc = nn.Linear(hidden, out_dim)

    def forward(self, seq):
        zeros = seq.new_zeros(self.layers, seq.shape[0], self.hidden)
        hseq, _ = self.lstm(seq, (zeros, zeros))
        return self.fc(hseq[:, -1, :])


class TorchFNN(nn.Module):
    """3 -> 50 -> 1 controller (Functions.py:239-289, width 1 so fc_int is idle)."""

    def __init__(self, in_dim=3, hidden=50, out_dim=1):
        super().__init__()
        self.fc_inp = nn.Linear(in_dim, hidden)
        self.fc_int = nn.Linear(hidden, hidden)
        self.fc_out = nn.Linear(hidden, out_dim, bias=False)

    def forward(self, x):
        return nn.functional.hardtanh(self.fc_out(torch.relu(self.fc_inp(x))))


def _con(xh):
    relu = torch.relu
    return relu(-xh[:, 1]) + relu(-xh[:, 2]) + relu(xh[:, 1] - P1_MAX) + relu(xh[:, 2] - P2_MAX)


def mpc_loss(sim, ctrl, X, u0, states, N, alpha, noise=None):
    """Rollout loss; u0 is (B,1) (the caller's ``controller(X)``), noise (B,N,4) or None.

    Returns (loss, feats) with feats = loss/command/error (B,), prediction (B*N,), xhat (B,N,4).
    """
    B = X.shape[0]
    ref = X[:, -1]
    window = states.clone()
    window[:, -1, -1] = u0.reshape(B)
    xh = sim(window)
    if noise is not None:
        xh = xh + noise[:, 0]
    err_terms = [torch.square(xh[:, 0] - ref)]
    cmd_terms = [alpha * torch.square(window[:, -2, -1] - window[:, -1, -1])]
    tot_terms = [err_terms[0] + cmd_terms[0] + _con(xh)]
    u_prev = u0.reshape(B, 1)
    preds = [u_prev]
    xhs = [xh]
    for j in range(1, N):
        u_next = ctrl(torch.stack((xh[:, 0], xh[:, 3], ref), dim=1))
        new_row = torch.cat((xh, u_next), dim=1).unsqueeze(1)
        window = torch.cat((window[:, 1:10, :], new_row), dim=1)
        xh = sim(window)
        if noise is not None:
            xh = xh + noise[:, j]
        err_terms.append(torch.square(xh[:, 0] - ref))
        cmd_terms.append(alpha * torch.square(u_prev.reshape(B) - u_next.reshape(B)))
        tot_terms.append(err_terms[-1] + cmd_terms[-1] + _con(xh))
        u_prev = u_next
        preds.append(u_next)
        xhs.append(xh)
    cost = torch.stack(tot_terms).sum(0) / N
    feats = {
        "loss": cost,
        "command": torch.stack(cmd_terms).sum(0) / N,
        "error": torch.stack(err_terms).sum(0) / N,
        "prediction": torch.cat(preds, dim=1).flatten(),
        "xhat": torch.stack(xhs, dim=1),
    }
    return cost.mean(), feats


def build_modules(params, dtype=torch.float32, lstm_requires_grad=True):
    """Instantiate TorchLSTM/TorchFNN from a NumPy param dict (see oracle.rollout_np)."""
    H = params["Whh"][0].shape[1]
    layers = len(params["Wih"])
    sim = TorchLSTM(params["Wih"][0].shape[1], H, params["fcW"].shape[0], layers).to(dtype)
    ctrl = TorchFNN(params["W_inp"].shape[1], params["W_inp"].shape[0], 1).to(dtype)
    with torch.no_grad():
        for l in range(layers):
            getattr(sim.lstm, f"weight_ih_l{l}").copy_(torch.as_tensor(params["Wih"][l]))
            getattr(sim.lstm, f"weight_hh_l{l}").copy_(torch.as_tensor(params["Whh"][l]))
        sim.fc.weight.copy_(torch.as_tensor(params["fcW"]))
        sim.fc.bias.copy_(torch.as_tensor(params["fcb"]))
        ctrl.fc_inp.weight.copy_(torch.as_tensor(params["W_inp"]))
        ctrl.fc_inp.bias.copy_(torch.as_tensor(params["b_inp"]))
        ctrl.fc_out.weight.copy_(torch.as_tensor(params["W_out"]))
    for p in sim.parameters():
        p.requires_grad_(lstm_requires_grad)
    return sim, ctrl


def loss_and_grads(params, X, u0, states, N, alpha, noise=None, dtype=torch.float32):
    """Run forward + ``loss.backward()`` exactly as train_model does (Functions.py:643-655).

    u0 enters as a leaf so its gradient (what autograd would hand the caller's controller(X) graph)
    is reported separately from the in-loss controller parameter gradients.
    Returns numpy dict: loss, feats..., g_u0, g_W_inp, g_b_inp, g_W_out.
    """
    sim, ctrl = build_modules(params, dtype)
    t = lambda a: torch.as_tensor(a, dtype=dtype)
    u0_t = t(u0).reshape(-1, 1).clone().requires_grad_(True)
    nz = None if noise is None else t(noise)
    loss, feats = mpc_loss(sim, ctrl, t(X), u0_t, t(states), N, alpha, nz)
    loss.backward()
    out = {k: v.detach().numpy() for k, v in feats.items()}
    out["loss_scalar"] = loss.detach().numpy()
    out["g_u0"] = u0_t.grad.reshape(-1).numpy()
    # N = 1: the controller is never called inside the loss, its grads stay None (== zero)
    g = lambda p: (p.grad if p.grad is not None else torch.zeros_like(p)).detach().numpy()
    out["g_W_inp"] = g(ctrl.fc_inp.weight)
    out["g_b_inp"] = g(ctrl.fc_inp.bias)
    out["g_W_out"] = g(ctrl.fc_out.weight)
    return out


def loss_and_grads_chunked(params, X, u0, states, N, alpha, noise=None, device="cpu", dtype=torch.float64,
                           chunk=16384):
    """:func:`loss_and_grads` for a large batch, evaluated chunk by chunk (on ``device``, e.g. the GPU in
    fp64: stock torch ops, the checker for full-size batches).

    Trajectories are independent until the batch mean (Functions.py:1463), so each chunk's loss is weighted
    by b_chunk / B and the parameter gradients summed over chunks are the full-batch gradients; per-
    trajectory outputs and g_u0 are concatenated. Inputs are arrays or tensors (any device); returns
    tensors on ``device`` in ``dtype``: loss (0-d), loss/command/error (B,), prediction (B*N,), xhat
    (B,N,4), g_u0 (B,), g_W_inp, g_b_inp, g_W_out.
    """
    sim, ctrl = build_modules(params, dtype, lstm_requires_grad=False)
    sim, ctrl = sim.to(device), ctrl.to(device)
    t = lambda a: torch.as_tensor(a).to(device=device, dtype=dtype)
    X, u0, states = t(X), t(u0).reshape(-1, 1), t(states)
    noise = None if noise is None else t(noise)
    B = X.shape[0]
    outs = {k: [] for k in ("loss", "command", "error", "prediction", "xhat", "g_u0")}
    total = torch.zeros((), dtype=dtype, device=device)
    for lo in range(0, B, chunk):
        hi = min(B, lo + chunk)
        u = u0[lo:hi].clone().requires_grad_(True)
        loss, f = mpc_loss(sim, ctrl, X[lo:hi], u, states[lo:hi], N, alpha, None if noise is None else noise[lo:hi])
        (loss * ((hi - lo) / B)).backward()
        total += loss.detach() * ((hi - lo) / B)
        for k in ("loss", "command", "error", "prediction", "xhat"):
            outs[k].append(f[k].detach())
        outs["g_u0"].append(u.grad.reshape(-1))
    out = {k: torch.cat(v) for k, v in outs.items()}
    out["loss_scalar"] = total
    g = lambda p: (p.grad if p.grad is not None else torch.zeros_like(p)).detach()
    out["g_W_inp"], out["g_b_inp"], out["g_W_out"] = g(ctrl.fc_inp.weight), g(ctrl.fc_inp.bias), g(ctrl.fc_out.weight)
    return out


def kink_margin(params, X, xhat):
    """Per-trajectory distance of the rollout's controller evaluations to the kinks of its piecewise-linear
    activations: min over horizon steps j >= 1 and hidden units of |z| (ReLU, Functions.py:276) and of
    |1 - |v|| (Hardtanh, :287), for the controller inputs [x̂_j[0], x̂_j[3], ref] of the fp64 trajectory
    ``xhat`` (B,N,4), and of the pressure predictions to the constraint ReLUs' kinks (0, P1_MAX, P2_MAX,
    :1411). Where an fp32 evaluation lands within its own rounding of a kink, its mask (and the
    gradient's slope there) can flip against fp64's: those trajectories' per-trajectory gradients differ by
    O(1) of one term, independent of the implementation's accuracy. Returns a (B,) fp64 tensor.
    """
    X = torch.as_tensor(X)
    xhat = torch.as_tensor(xhat).to(device=X.device, dtype=torch.float64)
    Wi = torch.as_tensor(params["W_inp"], dtype=torch.float64, device=X.device)
    bi = torch.as_tensor(params["b_inp"], dtype=torch.float64, device=X.device)
    Wo = torch.as_tensor(params["W_out"], dtype=torch.float64, device=X.device)
    B, N = xhat.shape[0], xhat.shape[1]
    # pressure-constraint ReLUs on every prediction (Functions.py:1411, 1449)
    p = xhat[..., 1:3]
    con = torch.minimum(p.abs(), (p - torch.tensor([P1_MAX, P2_MAX], dtype=torch.float64, device=X.device)).abs())
    con = con.amin(dim=(1, 2))
    if N < 2:
        return con
    ref = X[:, 2].to(torch.float64)
    cin = torch.stack((xhat[:, :-1, 0], xhat[:, :-1, 3], ref[:, None].expand(B, N - 1)), dim=-1)   # (B,N-1,3)
    z = cin @ Wi.T + bi
    v = torch.relu(z) @ Wo[0]
    return torch.minimum(con, torch.minimum(z.abs().amin(dim=(1, 2)), (1 - v.abs()).abs().amin(dim=1)))


def one_sided_g_u0(params, X, u0, states, N, alpha, rows, B_full, device="cpu", rel=(1e-9, 1e-8, 1e-7, 1e-6, 1e-5)):
    """The fp64 d loss / d u0 of trajectories ``rows`` of a batch of ``B_full`` trajectories, evaluated at u0 shifted
    by +-d for d in ``rel`` (absolute shifts of u0, a Hardtanh output in [-1, 1]): the one-sided derivatives on either
    side of a kink the trajectory passes near. Where an fp32 evaluation lands on the other side of such a kink than
    fp64 does (kink_margin), its g_u0 is — to fp32 accuracy — one of these values, not the fp64 value at u0: the
    full-size parity tests accept a kink-band trajectory above 1e-5 only when its g_u0 matches one of them
    (checker only). Returns {row: [(shift, g), ...]} with g in the full batch's units (the 1/B of the mean)."""
    t = lambda a: torch.as_tensor(a).to(device=device, dtype=torch.float64)
    X, u0, states = t(X), t(u0).reshape(-1), t(states)
    out = {}
    for r in rows:
        res = []
        for d in rel:
            for s in (d, -d):
                g = loss_and_grads_chunked(params, X[r:r + 1], (u0[r:r + 1] + s).reshape(1, 1), states[r:r + 1], N,
                                           alpha, device=device)["g_u0"]
                res.append((s, float(g[0]) / B_full))
        out[r] = res
    return out
