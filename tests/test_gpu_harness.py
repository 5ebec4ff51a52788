"""GPU: the reference's harness calls on the drop-in classes with the models on the device —
``predict`` / ``validate_model`` (Functions.py:679-748) through the HIP controller kernel, the surrogate step
(``simulator_make_step``, :969-1011) through the fused forward, and ``MPCLoss`` driven by duck-typed modules
shaped like the reference's own ``FNNModel`` / ``LSTMModel`` (not this package's classes)."""
import numpy as np
import pytest
import torch
from torch import nn

import forging_control_amd as fca
from conftest import load_case, relerr
from oracle import rollout_np as R
from test_harness import OUT_MAXABS, _loader, oracle_step, output_scaler, ref_lstm, windows

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 1e-5


def test_predict_and_validate_on_device():
    torch.manual_seed(5)
    ctrl = fca.FNNModel(3, 50, 1, 1).to(DEV)
    loader = _loader([15, 15, 7, 4096], 6)
    pred = fca.NeuralNetwork.predict(loader, ctrl)
    Wi, bi, Wo = (p.detach().cpu().double().numpy() for p in (ctrl.fc_inp.weight, ctrl.fc_inp.bias, ctrl.fc_out.weight))
    X = torch.cat([b[0] for b in loader]).double().numpy()
    u, _ = R.fnn_forward(X, Wi, bi, Wo)
    assert pred.is_cuda and pred.shape == (X.shape[0], 1)
    assert relerr(pred.cpu().numpy()[:, 0], u) <= TOL
    v = fca.NeuralNetwork.validate_model(loader, ctrl, nn.MSELoss(), DEV)
    off, exp = 0, []
    for Xb, yb, _ in loader:
        n = Xb.shape[0]
        exp.append(np.mean((u[off:off + n] - yb.double().numpy()[:, 0]) ** 2))
        off += n
    assert abs(v - np.mean(exp)) <= TOL * abs(np.mean(exp))


def test_simulator_make_step_on_device_matches_oracle():
    model, w = ref_lstm(DEV)
    sc = output_scaler()
    X = windows(300, 7)
    noise = np.random.default_rng(8).normal(0, 0.01, (300, 4))
    got = fca.NeuralNetwork.simulator_make_step(X, model, {"output": sc}, noise)
    exp = oracle_step(w, X, noise, sc)
    assert relerr(got / OUT_MAXABS, exp / OUT_MAXABS) <= TOL
    # the same model moved to the CPU (UL/Main.py:347-348) gives the same numbers through its own nn.LSTM
    got_cpu = fca.NeuralNetwork.simulator_make_step(X, model.to("cpu"), {"output": sc}, noise)
    assert relerr(got_cpu / OUT_MAXABS, got / OUT_MAXABS) <= TOL


class RefShapedFNN(nn.Module):
    """Attribute layout of the reference's FNNModel (Functions.py:239-289), not this package's class."""

    def __init__(self):
        super().__init__()
        self.width_dim = 1
        self.activation = nn.ReLU()
        self.constraint = nn.Hardtanh()
        self.fc_inp = nn.Linear(3, 50)
        self.fc_int = nn.Linear(50, 50)
        self.fc_out = nn.Linear(50, 1, bias=False)

    def forward(self, x):
        return self.constraint(self.fc_out(self.activation(self.fc_inp(x))))


class RefShapedLSTM(nn.Module):
    """Attribute layout of the reference's LSTMModel (Functions.py:317-379)."""

    def __init__(self):
        super().__init__()
        self.lstm = nn.LSTM(5, 50, 3, batch_first=True, bias=False)
        self.fc = nn.Linear(50, 4)


def test_mpcloss_accepts_reference_shaped_modules():
    c, params = load_case("ref_b256_n10")
    sim, ctrl = RefShapedLSTM(), RefShapedFNN()
    t = lambda a: torch.as_tensor(np.asarray(a, np.float32))
    with torch.no_grad():
        for k in range(3):
            getattr(sim.lstm, f"weight_ih_l{k}").copy_(t(params["Wih"][k]))
            getattr(sim.lstm, f"weight_hh_l{k}").copy_(t(params["Whh"][k]))
        sim.fc.weight.copy_(t(params["fcW"]))
        sim.fc.bias.copy_(t(params["fcb"]))
        ctrl.fc_inp.weight.copy_(t(params["W_inp"]))
        ctrl.fc_inp.bias.copy_(t(params["b_inp"]))
        ctrl.fc_out.weight.copy_(t(params["W_out"]))
    sim, ctrl = sim.to(DEV), ctrl.to(DEV)
    d = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=DEV)
    u0 = d(c["u0"]).reshape(-1, 1).requires_grad_(True)
    loss, f = fca.MPCLoss(c["N"], c["alpha"])(sim, ctrl, d(c["X"]), u0, d(c["states"]), DEV)
    loss.backward()
    assert abs(loss.item() - float(c["loss64"])) <= TOL * abs(float(c["loss64"]))
    assert relerr(f["prediction"].detach().cpu().numpy(), c["prediction_64"]) <= TOL
    assert relerr(u0.grad.reshape(-1).cpu().numpy(), c["g_u0_64"]) <= TOL
    assert relerr(ctrl.fc_inp.weight.grad.cpu().numpy(), c["g_W_inp_64"]) <= TOL
    assert relerr(ctrl.fc_out.weight.grad.cpu().numpy(), c["g_W_out_64"]) <= TOL
