"""LSTM surrogate training step: fcr_lstm_forward/backward vs the fp64 torch
restatement of Model_NN's train_model body (every weight gradient, the input gradient, AdamW steps)."""
import ctypes
import os

import numpy as np
import pytest
import torch

import forging_control_amd as fca
from conftest import GOLDEN, relerr
from oracle import surrogate_torch as S
from tests.golden.make_golden import synth_params

TOL = 1e-5


def ref_params():
    w = dict(np.load(os.path.join(GOLDEN, "weights_ref.npz")))
    return {"Wih": [w[f"Wih{k}"].astype(np.float64) for k in range(3)],
            "Whh": [w[f"Whh{k}"].astype(np.float64) for k in range(3)],
            "fcW": w["fcW"].astype(np.float64), "fcb": w["fcb"].astype(np.float64)}


def params_for(H, seed=0):
    if H == 50:
        return ref_params()
    p = synth_params(H, seed)
    return {"Wih": [np.asarray(a, np.float64) for a in p["Wih"]], "Whh": [np.asarray(a, np.float64) for a in p["Whh"]],
            "fcW": np.asarray(p["fcW"], np.float64), "fcb": np.asarray(p["fcb"], np.float64)}


def batch(B, seed):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-1, 1, (B, 10, 5))
    x[..., 1:3] = rng.uniform(0, 1.1, (B, 10, 2))      # pressures, as the rollout's windows
    return x, rng.uniform(-1, 1, (B, 4))


# ------------------------------------------------------------------------------------------------ CPU

def test_oracle_gradients_match_finite_differences():
    p = params_for(3, seed=1)
    x, target = batch(2, 0)
    _, loss, g = S.step_grads(p, x, target)
    rng = np.random.default_rng(0)
    for key, k in (("Wih", 0), ("Whh", 2), ("Wih", 1)):
        W = p[key][k]
        for _ in range(3):
            i = tuple(rng.integers(0, s) for s in W.shape)
            eps = 1e-6
            W[i] += eps
            lp = S.step_grads(p, x, target)[1]
            W[i] -= 2 * eps
            lm = S.step_grads(p, x, target)[1]
            W[i] += eps
            assert (lp - lm) / (2 * eps) == pytest.approx(g[key][k][i], rel=1e-6, abs=1e-10)


def test_lstm_model_on_cpu_is_its_own_nn_lstm():
    """Off the device the drop-in runs its own nn.LSTM + fc from a zero state (Functions.py:353-379), as the
    reference's closed-loop harness needs (model(X_new, "cpu"), Functions.py:999); the HIP entry refuses."""
    m = fca.LSTMModel(5, 50, 4, 3)
    x = torch.randn(2, 10, 5)
    zeros = torch.zeros(3, 2, 50)
    out, _ = m.lstm(x, (zeros, zeros))
    assert torch.equal(m(x, "cpu"), m.fc(out[:, -1, :]))
    with pytest.raises(RuntimeError, match="gfx950 LSTM path"):
        fca.surrogate.lstm_apply(m, x)


def test_abi_validates_before_any_device_call():
    lib = fca._native.load()
    d = fca.rollout.make_dims(16, 1, 50, 3, 1, 0.0)
    out = ctypes.c_size_t(0)
    assert lib.fcr_lstm_workspace_size(ctypes.byref(d), 1, ctypes.byref(out)) == 0
    fwd_only = ctypes.c_size_t(0)
    assert lib.fcr_lstm_workspace_size(ctypes.byref(d), 0, ctypes.byref(fwd_only)) == 0
    assert 0 < fwd_only.value < out.value
    bad = fca.rollout.make_dims(16, 1, 50, 2, 1, 0.0)
    assert lib.fcr_lstm_workspace_size(ctypes.byref(bad), 1, ctypes.byref(out)) == -4
    w = fca._native.FcrWeights()
    assert lib.fcr_lstm_forward(ctypes.byref(d), ctypes.byref(w), None, None, 1, None, 0, None) == -1
    assert "NULL" in lib.fcr_last_error().decode()
    assert lib.fcr_lstm_backward(ctypes.byref(d), ctypes.byref(w), None, None, None, None, None, None, None, 0,
                                 None) == -1


# ------------------------------------------------------------------------------------------------ GPU

def model_for(p, dev="cuda:0"):
    H = p["Whh"][0].shape[1]
    m = fca.LSTMModel(5, H, 4, 3).to(dev)
    t = lambda a: torch.as_tensor(np.asarray(a, np.float32))
    with torch.no_grad():
        for k in range(3):
            getattr(m.lstm, f"weight_ih_l{k}").copy_(t(p["Wih"][k]))
            getattr(m.lstm, f"weight_hh_l{k}").copy_(t(p["Whh"][k]))
        m.fc.weight.copy_(t(p["fcW"]))
        m.fc.bias.copy_(t(p["fcb"]))
    return m


def grads_of(m):
    return {"Wih": [getattr(m.lstm, f"weight_ih_l{k}").grad.cpu().numpy() for k in range(3)],
            "Whh": [getattr(m.lstm, f"weight_hh_l{k}").grad.cpu().numpy() for k in range(3)],
            "fcW": m.fc.weight.grad.cpu().numpy(), "fcb": m.fc.bias.grad.cpu().numpy()}


@pytest.mark.gpu
# H = 57: weight-gradient columns K % 8 != 0 (padded record tail); H = 256, B = 110: the W_hh reduction over 9 B rows
# takes more partial slices than the 10 B one (31 against 18: ADVICE r5, the partial slab is sized for both)
@pytest.mark.parametrize("H,B", [(50, 256), (50, 1), (50, 4099), (7, 33), (24, 1000), (64, 100), (256, 64), (256, 110),
                                 (96, 300), (264, 40), (57, 77)])
def test_gpu_training_step_matches_oracle(H, B):
    p = params_for(H, seed=H)
    x, target = batch(B, seed=B + H)
    y_ref, loss_ref, g_ref = S.step_grads(p, x, target)
    m = model_for(p)
    xt = torch.tensor(x, dtype=torch.float32, device="cuda:0", requires_grad=True)
    y = m(xt, "cuda:0")
    loss = torch.nn.functional.mse_loss(y, torch.tensor(target, dtype=torch.float32, device="cuda:0"))
    loss.backward()
    assert relerr(y.detach().cpu().numpy(), y_ref) < TOL
    assert abs(float(loss) - loss_ref) <= TOL * abs(loss_ref)
    g = grads_of(m)
    for key in ("Wih", "Whh"):
        for k in range(3):
            assert relerr(g[key][k], g_ref[key][k]) < TOL, (key, k, relerr(g[key][k], g_ref[key][k]))
    assert relerr(g["fcW"], g_ref["fcW"]) < TOL and relerr(g["fcb"], g_ref["fcb"]) < TOL
    assert relerr(xt.grad.cpu().numpy(), g_ref["x"]) < TOL


@pytest.mark.gpu
def test_gpu_adamw_trajectory_matches_oracle():
    """Five train_model iterations (MSE + AdamW lr 1e-3, wd 0; Model_NN/Main.py:229-232) on fixed batches:
    the parameters after the last step agree with the fp64 restatement."""
    p = ref_params()
    batches = [batch(256, seed=s) for s in range(5)]
    ref, ref_losses = S.train_steps(p, batches, lr=1e-3)
    m = model_for(p)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=0.0)
    loader = [(torch.tensor(x, dtype=torch.float32), torch.tensor(t, dtype=torch.float32)) for x, t in batches]
    losses = []
    for X, Y in loader:           # fca.surrogate.train_model's body, losses kept per step
        X, Y = X.to("cuda:0"), Y.to("cuda:0")
        opt.zero_grad()
        loss = torch.nn.functional.mse_loss(m(X, "cuda:0"), Y.squeeze())
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert np.allclose(losses, ref_losses, rtol=TOL)
    got = {"Wih": [getattr(m.lstm, f"weight_ih_l{k}").detach().cpu().numpy() for k in range(3)],
           "Whh": [getattr(m.lstm, f"weight_hh_l{k}").detach().cpu().numpy() for k in range(3)]}
    for key in ("Wih", "Whh"):
        for k in range(3):
            assert relerr(got[key][k], ref[key][k]) < TOL
    avg = fca.surrogate.train_model(loader, m, torch.nn.MSELoss(), opt, "cuda:0")
    assert np.isfinite(avg)


@pytest.mark.gpu
def test_gpu_forward_matches_rollout_kernel_one_step():
    """The surrogate forward and the rollout's first LSTM call (fused kernel, N = 1) agree on a window."""
    p = ref_params()
    x, _ = batch(512, seed=3)
    m = model_for(p)
    xt = torch.tensor(x, dtype=torch.float32, device="cuda:0")
    with torch.no_grad():
        y = m(xt, "cuda:0")
    y2 = fca.simulate_step(m, xt)
    assert relerr(y.cpu().numpy(), y2.cpu().numpy()) < 2 * TOL


def _oracle_grads_dy(p, x, dy, dev):
    """fp64 autograd of y = LSTMModel(x) against an arbitrary dL/dy (the oracle model on `dev`)."""
    m = S.build(p).to(dev)
    xt = torch.as_tensor(x, dtype=torch.float64, device=dev).clone().requires_grad_(True)
    y = m(xt)
    y.backward(torch.as_tensor(dy, dtype=torch.float64, device=dev))
    g = {"Wih": [getattr(m.lstm, f"weight_ih_l{k}").grad.cpu().numpy() for k in range(3)],
         "Whh": [getattr(m.lstm, f"weight_hh_l{k}").grad.cpu().numpy() for k in range(3)],
         "fcW": m.fc.weight.grad.cpu().numpy(), "fcb": m.fc.bias.grad.cpu().numpy(), "x": xt.grad.cpu().numpy()}
    return y.detach().cpu().numpy(), g


def _hip_grads_dy(p, x, dy):
    m = model_for(p)
    xt = torch.tensor(x, dtype=torch.float32, device="cuda:0", requires_grad=True)
    y = m(xt, "cuda:0")
    y.backward(torch.tensor(dy, dtype=torch.float32, device="cuda:0"))
    g = grads_of(m)
    g["x"] = xt.grad.cpu().numpy()
    return y.detach().cpu().numpy(), g


def _check_all(y, g, y_ref, g_ref, tol=TOL):
    assert relerr(y, y_ref) < tol
    for key in ("Wih", "Whh"):
        for k in range(3):
            assert relerr(g[key][k], g_ref[key][k]) < tol, (key, k, relerr(g[key][k], g_ref[key][k]))
    for key in ("fcW", "fcb", "x"):
        assert relerr(g[key], g_ref[key]) < tol, (key, relerr(g[key], g_ref[key]))


@pytest.mark.gpu
def test_gpu_full_batch_step_matches_oracle():
    """B = 65 536 (the benchmark's batch), H = 50: every weight gradient summed over 655 360 (window, step) rows, the
    readout's over 65 536 windows, and dL/dx, against fp64 autograd (on the GPU, checker only)."""
    p = ref_params()
    x, target = batch(65536, seed=7)
    B = x.shape[0]
    dy = 2.0 * (0.0 + 1.0) / (B * 4) * np.random.default_rng(8).uniform(-1, 1, (B, 4))   # an MSE-sized dL/dy
    y_ref, g_ref = _oracle_grads_dy(p, x, dy, "cuda:0")
    y, g = _hip_grads_dy(p, x, dy)
    _check_all(y, g, y_ref, g_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("H", [50, 256])
def test_gpu_rows_without_or_with_tiny_gradient(H):
    """Per-row dgate scales: windows with dL/dy = 0, ~1e-30 and ~1e4 in one batch (H <= 52: the weight-gradient kernel
    rescales every row to its workgroup's largest, and zero rows must not set that scale; H > 52: the fused backward
    cells' per-row powers of two, and the fp32 weight-gradient reductions)."""
    p = ref_params() if H == 50 else params_for(H, seed=H)
    x, _ = batch(4099, seed=11)
    rng = np.random.default_rng(12)
    dy = rng.uniform(-1, 1, (4099, 4))
    dy[::3] = 0.0
    dy[1::7] *= 1e-30
    dy[5::11] *= 1e4
    y_ref, g_ref = _oracle_grads_dy(p, x, dy, "cuda:0")
    y, g = _hip_grads_dy(p, x, dy)
    _check_all(y, g, y_ref, g_ref)
    # the tiny rows alone: their gradients are not flushed (every row's own power-of-two scale)
    dt = np.zeros_like(dy)
    dt[1::7] = dy[1::7]
    _, gt_ref = _oracle_grads_dy(p, x, dt, "cuda:0")
    _, gt = _hip_grads_dy(p, x, dt)
    for key in ("Wih", "Whh"):
        for k in range(3):
            assert relerr(gt[key][k], gt_ref[key][k]) < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("H", [50, 96])
def test_gpu_range_guarded_window_columns(H):
    """Unscaled window columns (|x| up to 3e4 and 1e5, beyond f16's range: hi = f16(x) would be inf): the range guard
    (fcr_pack.h) runs them on x 2^-s_c against W_ih0 2^s_c and scales their weight gradients back. Against O(1) weights
    the layer-0 gates cancel terms of ~1e4, where any fp32 implementation is off fp64 by ~|W||x| 2^-24 (stock torch
    fp32: 4e-4 on W_ih0's gradient here) — so, as the rollout's test of the guard (test_gpu_parity.py), every tensor is
    held to max(1e-5, 4 x torch fp32's own distance to fp64). H = 96: the wide path's window records carry the guard."""
    p = ref_params() if H == 50 else params_for(H, seed=H)
    x, target = batch(300, seed=13)
    x[..., 0] *= 3e4
    x[..., 4] *= 1e5
    dy = np.random.default_rng(14).uniform(-1, 1, (300, 4)) * 1e-3
    y_ref, g_ref = _oracle_grads_dy(p, x, dy, "cuda:0")
    m32 = S.build(p, torch.float32)
    xt = torch.as_tensor(x, dtype=torch.float32).clone().requires_grad_(True)
    y32 = m32(xt)
    y32.backward(torch.as_tensor(dy, dtype=torch.float32))
    g32 = {"Wih": [getattr(m32.lstm, f"weight_ih_l{k}").grad.numpy() for k in range(3)],
           "Whh": [getattr(m32.lstm, f"weight_hh_l{k}").grad.numpy() for k in range(3)],
           "fcW": m32.fc.weight.grad.numpy(), "fcb": m32.fc.bias.grad.numpy(), "x": xt.grad.numpy()}
    y, g = _hip_grads_dy(p, x, dy)
    assert np.isfinite(y).all() and relerr(y, y_ref) <= max(TOL, 4 * relerr(y32.detach().numpy(), y_ref))
    pairs = [(g[k][i], g32[k][i], g_ref[k][i]) for k in ("Wih", "Whh") for i in range(3)]
    pairs += [(g[k], g32[k], g_ref[k]) for k in ("fcW", "fcb", "x")]
    for got, t32, ref in pairs:
        assert np.isfinite(got).all()
        assert relerr(got, ref) <= max(TOL, 4 * relerr(t32, ref)), (relerr(got, ref), relerr(t32, ref))
