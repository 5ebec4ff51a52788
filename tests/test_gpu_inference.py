"""GPU: batched one-step LSTM inference (simulator_make_step, Functions.py:969-1011) on the rollout
kernel, against the fp64 oracle's LSTM forward (oracle/rollout_np.py lstm_forward)."""
import numpy as np
import pytest
import torch

import forging_control_amd as fca
from conftest import load_case, relerr
from oracle import rollout_np as R
from test_gpu_parity import modules

pytestmark = pytest.mark.gpu


def _windows(B, seed):
    g = np.random.default_rng(seed)
    w = np.empty((B, 10, 5))
    w[..., [0, 3, 4]] = g.uniform(-1, 1, (B, 10, 3))
    w[..., 1:3] = g.uniform(0, 1.1, (B, 10, 2))
    return w.astype(np.float32)


def _oracle(params, w, noise=None):
    y, _ = R.lstm_forward(w.astype(np.float64), params["Wih"], params["Whh"], params["fcW"], params["fcb"])
    return y + (0 if noise is None else noise)


@pytest.mark.parametrize("case,B", [("ref_b15_n10", 1), ("ref_b15_n10", 1000), ("h256_b8_n25", 40)])
def test_simulate_step_matches_oracle(case, B):
    params = load_case(case)[1]
    sim, _ = modules(params)
    w = _windows(B, 3 + B)
    nz = np.random.default_rng(B).standard_normal((B, 4)).astype(np.float32) * 0.01
    got = fca.simulate_step(sim, torch.as_tensor(w, device="cuda"), torch.as_tensor(nz, device="cuda"))
    assert relerr(got.cpu().numpy(), _oracle(params, w, nz)) <= 1e-5


def test_simulator_make_step_dropin_unscales():
    class MaxAbs:   # the reference's scalers are sklearn MaxAbsScaler: inverse_transform = x * max_abs_
        max_abs_ = np.array([0.9113443, 1.50775144e7, 3.08810905e7, 0.3758976])

        def inverse_transform(self, y):
            return y * self.max_abs_

    params = load_case("ref_b15_n10")[1]
    sim, _ = modules(params)
    w = _windows(1, 11)
    nz = np.array([0.01, -0.02, 0.0, 0.005], np.float32)
    out = fca.simulator_make_step(w, sim, {"output": MaxAbs()}, nz)
    assert out.shape == (1, 4)
    assert relerr(out, _oracle(params, w, nz) * MaxAbs.max_abs_) <= 1e-5
