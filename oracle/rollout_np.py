"""fp64 NumPy restatement of the unsupervised-MPC rollout loss with a hand-written reverse pass.

TEST INFRASTRUCTURE ONLY. Nothing in the product package imports this module; only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use it, and only as the
checker.

PARITY STATUS: *parity unpinned*. The reference (marcowus/forging-control) ships no tests, fixtures
or golden vectors for this path, and executing its Python was denied by the
environment. This restatement is pinned instead against a second, independent
restatement (``oracle/rollout_torch.py``: stock ``torch.nn.LSTM`` + autograd, same op order as the
reference) to ~1e-12 in fp64, and the committed fixtures in ``tests/golden/`` use the reference's own
trained weights (``Model_NN/results/model_NN.pt``, ``results/NN_controller_N_10_0.pt``) loaded as data.

What it restates (all paths relative to ``/root/reference/Unsupervised Learning/``):

* ``MPCLoss.forward``            Functions.py:1353-1472  -> :func:`rollout_forward`
* ``LSTMModel.forward``          Functions.py:353-379    -> :func:`lstm_forward`
  (``nn.LSTM(5, H, 3, batch_first=True, bias=False)`` from zero state, gate order i|f|g|o, then
  ``fc`` on the last step, Functions.py:325-329)
* ``FNNModel.forward``           Functions.py:261-289    -> :func:`fnn_forward`
  (Linear+ReLU, Linear without bias, Hardtanh[-1, 1]; width 1 so ``fc_int`` is never applied)
* ``loss.backward()``            Functions.py:655        -> :func:`rollout_backward`
  (only the gradients the optimizer consumes: controller parameters and ``u0``; the reference also
  computes LSTM weight gradients that nothing reads)
"""
from __future__ import annotations

import numpy as np

# Pressure-constraint upper bounds, Functions.py:1411 and :1449 (32e6 / scaler max_abs_).
P1_MAX = 2.122366
P2_MAX = 1.036233


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


# ---------------------------------------------------------------------------------------------
# FNN controller (Functions.py:239-289)
# ---------------------------------------------------------------------------------------------
def fnn_forward(x, W_inp, b_inp, W_out):
    """u = Hardtanh(W_out · ReLU(W_inp · x + b_inp)); x (B,3) -> u (B,), plus the cache."""
    z = x @ W_inp.T + b_inp            # fc_inp, Functions.py:275
    a = np.maximum(z, 0.0)             # ReLU,   Functions.py:276
    v = a @ W_out[0]                   # fc_out (no bias), Functions.py:284
    u = np.clip(v, -1.0, 1.0)          # Hardtanh, Functions.py:287
    return u, (x, z, a, v)


def fnn_backward(du, cache, W_inp, W_out):
    """Reverse of :func:`fnn_forward` with torch's kink conventions.

    Hardtanh'(v) = 1[-1 < v < 1] (ATen hardtanh_backward), ReLU'(z) = 1[z > 0] (threshold_backward).
    Returns (dx (B,3), dW_inp, db_inp, dW_out) with the parameter grads summed over the batch.
    """
    x, z, a, v = cache
    dv = du * ((v > -1.0) & (v < 1.0))
    dW_out = (dv[:, None] * a).sum(0)[None, :]
    da = dv[:, None] * W_out[0][None, :]
    dz = da * (z > 0.0)
    dW_inp = dz.T @ x
    db_inp = dz.sum(0)
    dx = dz @ W_inp
    return dx, dW_inp, db_inp, dW_out


# ---------------------------------------------------------------------------------------------
# LSTM surrogate (Functions.py:317-379; torch.nn.LSTM semantics)
# ---------------------------------------------------------------------------------------------
def lstm_forward(win, Wih, Whh, fcW, fcb):
    """Stacked LSTM from h=c=0 over win (B,L,5); returns (out (B,4), cache)."""
    B, L, _ = win.shape
    x = win
    cache = []
    for l in range(len(Wih)):
        H = Whh[l].shape[1]
        h = np.zeros((B, H))
        c = np.zeros((B, H))
        hs, cells = [], []
        for t in range(L):
            g = x[:, t] @ Wih[l].T + h @ Whh[l].T
            i = _sig(g[:, 0:H])
            f = _sig(g[:, H:2 * H])
            gg = np.tanh(g[:, 2 * H:3 * H])
            o = _sig(g[:, 3 * H:4 * H])
            c_prev = c
            c = f * c + i * gg
            tc = np.tanh(c)
            h = o * tc
            cells.append((i, f, gg, o, c_prev, tc))
            hs.append(h)
        cache.append(cells)
        x = np.stack(hs, axis=1)
    out = x[:, -1] @ fcW.T + fcb                  # fc on last step, Functions.py:377
    return out, cache


def lstm_backward(dout, cache, Wih, Whh, fcW, in_dim):
    """Input gradient of :func:`lstm_forward` (LSTM weight grads are skipped on purpose)."""
    B = dout.shape[0]
    L = len(cache[0])
    H_top = Whh[-1].shape[1]
    dseq = np.zeros((B, L, H_top))
    dseq[:, L - 1] = dout @ fcW
    for l in reversed(range(len(Wih))):
        H = Whh[l].shape[1]
        d_in = np.zeros((B, L, Wih[l].shape[1]))
        dh_next = np.zeros((B, H))
        dc_next = np.zeros((B, H))
        for t in reversed(range(L)):
            i, f, gg, o, c_prev, tc = cache[l][t]
            dh = dseq[:, t] + dh_next
            dc = dc_next + dh * o * (1.0 - tc * tc)
            dgates = np.concatenate([
                dc * gg * i * (1.0 - i),
                dc * c_prev * f * (1.0 - f),
                dc * i * (1.0 - gg * gg),
                dh * tc * o * (1.0 - o),
            ], axis=1)
            d_in[:, t] = dgates @ Wih[l]
            dh_next = dgates @ Whh[l]
            dc_next = dc * f
        dseq = d_in
    assert dseq.shape[2] == in_dim
    return dseq


# ---------------------------------------------------------------------------------------------
# Rollout (MPCLoss.forward, Functions.py:1353-1472)
# ---------------------------------------------------------------------------------------------
def _constraint(xh):
    """ReLU(-p1) + ReLU(-p2) + ReLU(p1 - P1_MAX) + ReLU(p2 - P2_MAX), Functions.py:1411."""
    p1, p2 = xh[:, 1], xh[:, 2]
    return (np.maximum(-p1, 0.0) + np.maximum(-p2, 0.0)
            + np.maximum(p1 - P1_MAX, 0.0) + np.maximum(p2 - P2_MAX, 0.0))


def _constraint_grad(xh):
    p1, p2 = xh[:, 1], xh[:, 2]
    g = np.zeros_like(xh)
    g[:, 1] = -1.0 * (-p1 > 0) + 1.0 * (p1 - P1_MAX > 0)
    g[:, 2] = -1.0 * (-p2 > 0) + 1.0 * (p2 - P2_MAX > 0)
    return g


def rollout_forward(params, X, u0, states, N, alpha, noise=None):
    """Forward rollout. Returns (loss, feats, tape).

    params: dict with W_inp (50,3), b_inp (50,), W_out (1,50), Wih [3], Whh [3], fcW (4,H), fcb (4,)
    X (B,3) = [y_dot, z, ref]; u0 (B,) = controller(X); states (B,10,5); noise (B,N,4) or None.
    feats: loss (B,), command (B,), error (B,), prediction (B*N,) sample-major, xhat (B,N,4).
    """
    X = np.asarray(X, np.float64)
    states = np.asarray(states, np.float64)
    u0 = np.asarray(u0, np.float64).reshape(-1)
    B = X.shape[0]
    ref = X[:, -1]                                             # Functions.py:1392
    win = states.copy()
    win[:, -1, -1] = u0                                        # Functions.py:1395-1396
    Wih, Whh, fcW, fcb = params["Wih"], params["Whh"], params["fcW"], params["fcb"]
    xh, lcache = lstm_forward(win, Wih, Whh, fcW, fcb)         # Functions.py:1399
    if noise is not None:
        xh = xh + noise[:, 0]                                  # Functions.py:1400-1402
    cmd = np.zeros((N, B))
    err = np.zeros((N, B))
    con = np.zeros((N, B))
    cmd[0] = alpha * (win[:, -2, -1] - win[:, -1, -1]) ** 2   # Functions.py:1405
    err[0] = (xh[:, 0] - ref) ** 2                             # Functions.py:1408
    con[0] = _constraint(xh)                                   # Functions.py:1411
    us = [u0]
    xhs = [xh]
    lcaches = [lcache]
    fcaches = []
    wins = [win]
    for j in range(N - 1):                                     # Functions.py:1421
        cin = np.stack([xh[:, 0], xh[:, 3], ref], axis=1)      # Functions.py:1424
        u_new, fc_ = fnn_forward(cin, params["W_inp"], params["b_inp"], params["W_out"])
        row = np.concatenate([xh, u_new[:, None]], axis=1)[:, None, :]
        win = np.concatenate([win[:, 1:10, :], row], axis=1)   # Functions.py:1433-1434
        xh, lcache = lstm_forward(win, Wih, Whh, fcW, fcb)     # Functions.py:1437
        if noise is not None:
            xh = xh + noise[:, j + 1]
        err[j + 1] = (xh[:, 0] - ref) ** 2                     # Functions.py:1443
        cmd[j + 1] = alpha * (us[-1] - u_new) ** 2             # Functions.py:1446
        con[j + 1] = _constraint(xh)                           # Functions.py:1449
        us.append(u_new)
        xhs.append(xh)
        lcaches.append(lcache)
        fcaches.append(fc_)
        wins.append(win)
    cost = (err + cmd + con).sum(0) / N                        # Functions.py:1458
    feats = {
        "loss": cost,
        "command": cmd.sum(0) / N,                             # Functions.py:1459
        "error": err.sum(0) / N,                               # Functions.py:1460
        "prediction": np.stack(us, axis=1).reshape(-1),        # Functions.py:1466
        "xhat": np.stack(xhs, axis=1),
    }
    loss = cost.mean()                                         # Functions.py:1463
    tape = dict(B=B, N=N, alpha=alpha, ref=ref, us=us, xhs=xhs, lcaches=lcaches,
                fcaches=fcaches, s84=states[:, 8, 4].astype(np.float64))
    return loss, feats, tape


def rollout_backward(params, tape, dloss=1.0):
    """Reverse pass of :func:`rollout_forward`.

    Returns dict with g_u0 (B,), g_W_inp (50,3), g_b_inp (50,), g_W_out (1,50) — the gradients that
    ``loss.backward()`` (Functions.py:655) delivers to the caller's ``controller(X)`` graph (via u0)
    and to the controller parameters used inside the loss.
    """
    B, N, alpha, ref = tape["B"], tape["N"], tape["alpha"], tape["ref"]
    us, xhs = tape["us"], tape["xhs"]
    Wih, Whh, fcW = params["Wih"], params["Whh"], params["fcW"]
    W_inp, W_out = params["W_inp"], params["W_out"]
    w = dloss / (B * N)                        # d loss / d (each per-step cost term)
    # Gradient accumulators for the generated window rows E[10+i] = (xhat_i, u_{i+1}).
    G = np.zeros((max(N - 1, 0), B, 5))
    g_u0 = np.zeros(B)
    du = [np.zeros(B) for _ in range(N)]       # du[k] = d loss / d u_k (direct cost terms)
    # command cost terms: cmd_0 = a(s84 - u0)^2, cmd_k = a(u_{k-1} - u_k)^2
    du[0] += w * 2.0 * alpha * (us[0] - tape["s84"])
    for k in range(1, N):
        dd = w * 2.0 * alpha * (us[k - 1] - us[k])
        du[k - 1] += dd
        du[k] -= dd
    g_W_inp = np.zeros_like(W_inp)
    g_b_inp = np.zeros(W_inp.shape[0])
    g_W_out = np.zeros_like(W_out)
    for j in reversed(range(N)):
        dxh = np.zeros((B, 4))
        dxh[:, 0] += w * 2.0 * (xhs[j][:, 0] - ref)
        dxh += w * _constraint_grad(xhs[j])
        if j <= N - 2:
            dxh += G[j][:, 0:4]
            du_next = du[j + 1] + G[j][:, 4]
            dcin, dWi, dbi, dWo = fnn_backward(du_next, tape["fcaches"][j], W_inp, W_out)
            g_W_inp += dWi
            g_b_inp += dbi
            g_W_out += dWo
            dxh[:, 0] += dcin[:, 0]
            dxh[:, 3] += dcin[:, 1]
        dwin = lstm_backward(dxh, tape["lcaches"][j], Wih, Whh, fcW, 5)   # (B,10,5)
        L = dwin.shape[1]
        for t in range(L):
            rowid = j + t                      # extended-sequence row index
            if rowid >= 10:
                G[rowid - 10] += dwin[:, t]
            elif rowid == 9:
                g_u0 += dwin[:, t, 4]
    g_u0 += du[0]
    return {"g_u0": g_u0, "g_W_inp": g_W_inp, "g_b_inp": g_b_inp, "g_W_out": g_W_out}


def adamw_step(p, g, m, v, step, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, wd=1e-2):
    """torch.optim.AdamW (defaults except lr, UL/Main.py:195), one step, in place on copies."""
    p = p * (1.0 - lr * wd)
    m = betas[0] * m + (1.0 - betas[0]) * g
    v = betas[1] * v + (1.0 - betas[1]) * g * g
    bc1 = 1.0 - betas[0] ** step
    bc2 = 1.0 - betas[1] ** step
    p = p - lr * (m / bc1) / (np.sqrt(v / bc2) + eps)
    return p, m, v
