"""CPU: the oracle restatements against each other and against the committed golden fixtures."""
import numpy as np
import pytest
import torch

from conftest import relerr
from oracle import rollout_np as R
from oracle import rollout_torch as T

FEATS = ("loss", "command", "error", "prediction", "xhat")
GRADS = ("g_u0", "g_W_inp", "g_b_inp", "g_W_out")


def test_numpy_oracle_reproduces_golden_fp64(golden):
    name, c, params = golden
    nz = None if c["noise"] is None else c["noise"].astype(np.float64)
    loss, feats, tape = R.rollout_forward(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"], nz)
    g = R.rollout_backward(params, tape)
    assert abs(loss - float(c["loss64"])) <= 1e-12 * max(1.0, abs(loss))
    for k in FEATS:
        assert relerr(feats[k], c[f"{k}_64"]) < 1e-12, k
    for k in GRADS:
        assert relerr(g[k], c[f"{k}_64"]) < 1e-12, k


def test_torch_oracle_fp64_agrees_with_numpy(golden):
    name, c, params = golden
    if c["B"] > 64:
        pytest.skip("large case covered by the fp64 golden check")
    o = T.loss_and_grads(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"], c["noise"], dtype=torch.float64)
    for k in FEATS:
        assert relerr(o[k], c[f"{k}_64"]) < 1e-10, k
    for k in GRADS:
        assert relerr(o[k], c[f"{k}_64"]) < 1e-10, k


def test_fp32_reference_within_1e5_of_fp64(golden):
    """The tolerance the GPU path is held to is meaningful: torch fp32 itself sits ~1e-6 from fp64."""
    name, c, params = golden
    for k in FEATS + GRADS:
        assert relerr(c[f"{k}_32"], c[f"{k}_64"]) < 1e-5, k


def test_stress_fixtures_cover_branches():
    from conftest import load_case
    c, _ = load_case("ref_wide_b64_n10")
    assert c["con_active"] > 0 and c["u_saturated"] > 0     # constraint ReLUs and Hardtanh clamp fire
    c, _ = load_case("h16_b33_n4")
    assert c["con_active"] > 0


def test_noise_is_additive_after_lstm():
    """Functions.py:1400-1402: noise shifts xhat but the costs use the noisy value."""
    from conftest import load_case
    c, params = load_case("refnoise_b15_n10")
    _, f0, _ = R.rollout_forward(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"], None)
    _, f1, _ = R.rollout_forward(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"], c["noise"].astype(np.float64))
    d = f1["xhat"][:, 0] - f0["xhat"][:, 0]
    assert np.allclose(d, c["noise"][:, 0], atol=1e-12)


def test_adamw_restatement_matches_torch():
    p = np.linspace(-1, 1, 7)
    g = np.cos(np.arange(7.0))
    tp = torch.nn.Parameter(torch.tensor(p))
    opt = torch.optim.AdamW([tp], lr=1e-4)
    m = np.zeros(7)
    v = np.zeros(7)
    q = p.copy()
    for step in range(1, 4):
        tp.grad = torch.tensor(g * step)
        opt.step()
        q, m, v = R.adamw_step(q, g * step, m, v, step)
    assert np.allclose(tp.detach().numpy(), q, rtol=0, atol=1e-15)
