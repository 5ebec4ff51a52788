"""Full-size parity at the benchmarked batch sizes (BASELINE.json configs 2, 3 and 5): the gfx950 rollout's
loss, per-trajectory features, x̂, per-trajectory u0 gradients AND the controller-parameter gradients —
sums over all B·N (trajectory, step) terms — against the stock-torch restatement (oracle/rollout_torch.py)
evaluated in fp64 on the same GPU, chunked over trajectories (independent until the batch mean,
Functions.py:1463; each chunk's loss weighted by b_chunk / B). Metric: per tensor max|hip - ref| / max|ref|
(SURVEY.md §8(d)); parity unpinned (no reference output exists at these sizes)."""
import numpy as np
import pytest
import torch

import forging_control_amd as fca
from oracle import rollout_torch as T
from tests.golden.make_golden import synth_inputs, synth_params
import test_gpu_parity as P
from conftest import load_case

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
PER_TRAJ = ("loss", "command", "error", "prediction", "xhat", "g_u0")
PARAMS = ("g_W_inp", "g_b_inp", "g_W_out")
# kink band: trajectories whose fp64 rollout passes within DELTA of a ReLU / Hardtanh / constraint kink
# (oracle.rollout_torch.kink_margin) can have an fp32 mask flipped against fp64 — an O(1) change of one
# term's slope that any fp32 implementation shows (torch's own fp32 path included); at B·N ~ 10^6 a few
# trajectories always do. They are compared separately, and the parameter sums re-checked without them.
DELTA = 1e-5


def _hip(params, Xd, Sd, N, precision):
    sim, ctrl = P.modules(params)
    with torch.no_grad():
        u0 = ctrl(Xd)
    u = u0.clone().requires_grad_(True)
    fn = fca.MPCLoss(prediction_horizon=N, alpha=20.0, precision=precision)
    loss, f = fn(sim, ctrl, Xd, u, Sd, DEV)
    loss.backward()
    got = {k: v.detach() for k, v in f.items()}
    got["prediction"] = got["prediction"].reshape(Xd.shape[0], N)
    got["xhat"] = fn.last_trajectory
    got["g_u0"] = u.grad.reshape(-1)
    got["g_W_inp"], got["g_b_inp"], got["g_W_out"] = ctrl.fc_inp.weight.grad, ctrl.fc_inp.bias.grad, ctrl.fc_out.weight.grad
    got["loss_scalar"] = loss.detach()
    del fn, loss, f
    torch.cuda.empty_cache()
    return got, u.detach()


def _err(a, r, rows=None):
    a, r = a.double(), r.reshape(a.shape)
    if rows is not None:
        a, r = a[rows], r[rows]
    return float((a - r).abs().max() / r.abs().max())


def hip_and_oracle(params, B, N, seed, precision="fp32", chunk=16384):
    """Returns (err, info): err holds per-trajectory errors over the trajectories outside the kink band,
    parameter-gradient errors of the full batch ('<g>_full') and of the batch without the kink-band
    trajectories (re-run on the GPU and the oracle: '<g>'), and the loss."""
    X, S, _ = synth_inputs(B, N, seed)
    d = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=DEV)
    Xd, Sd = d(X), d(S)
    got, u0 = _hip(params, Xd, Sd, N, precision)
    ref = T.loss_and_grads_chunked(params, Xd, u0, Sd, N, 20.0, device=DEV, chunk=chunk)
    reg = T.kink_margin(params, Xd.double(), ref["xhat"].reshape(B, N, 4)) > DELTA
    err = {k: _err(got[k], ref[k], reg) for k in PER_TRAJ}
    err.update({f"{k}_full": _err(got[k], ref[k]) for k in PARAMS})
    err["loss_scalar"] = _err(got["loss_scalar"], ref["loss_scalar"])
    kink = (~reg).nonzero().reshape(-1)
    info = {"kink_trajectories": int(kink.numel()),
            "g_u0_err_in_kink_band": _err(got["g_u0"], ref["g_u0"], ~reg) if kink.numel() else 0.0}
    del got, ref
    idx = reg.nonzero().reshape(-1)
    sub, u_sub = _hip(params, Xd[idx].contiguous(), Sd[idx].contiguous(), N, precision)
    ref = T.loss_and_grads_chunked(params, Xd[idx], u_sub, Sd[idx], N, 20.0, device=DEV, chunk=chunk)
    err.update({k: _err(sub[k], ref[k]) for k in PARAMS})
    print({k: f"{v:.2e}" for k, v in err.items()}, info)
    return err, info


def _check(err, info, B, tol_traj, tol_gu0, tol_grad, tol_loss):
    assert info["kink_trajectories"] <= 0.05 * B, info
    assert err["loss_scalar"] <= tol_loss, err
    assert max(err[k] for k in PER_TRAJ if k != "g_u0") <= tol_traj, err
    assert err["g_u0"] <= tol_gu0, err
    assert max(err[k] for k in PARAMS) <= tol_grad, err
    # the kink-band flips move the full-batch parameter sums by a few terms out of B·N
    assert max(err[f"{k}_full"] for k in PARAMS) <= 10 * tol_grad, err


@pytest.fixture(scope="module")
def ref_params():
    return load_case("ref_b15_n10")[1]


def test_config2_full_batch_parameter_gradients(ref_params):
    """B = 65 536, N = 10, H = 50, fp32: every output and the controller gradients summed over 655 360 terms."""
    _check(*hip_and_oracle(ref_params, 65536, 10, 21), 65536, 1e-5, 1e-5, 1e-5, 1e-5)


def test_config3_full_batch_fp32(ref_params):
    """B = 262 144 in the default fp32-accurate mode."""
    _check(*hip_and_oracle(ref_params, 262144, 10, 22), 262144, 1e-5, 1e-5, 1e-5, 1e-5)


def test_config3_full_batch_f16fwd(ref_params):
    """B = 262 144 in config 3's mode (f16 forward, fp32-accurate backward) at the stated tolerances
    (tests/test_gpu_precision.py)."""
    from test_gpu_precision import TOL_FEATS, TOL_GRADS_F16FWD_FULL, TOL_GU0_F16FWD, TOL_LOSS
    _check(*hip_and_oracle(ref_params, 262144, 10, 23, precision="f16fwd"), 262144, TOL_FEATS, TOL_GU0_F16FWD,
           TOL_GRADS_F16FWD_FULL, TOL_LOSS)


def test_config5_full_batch():
    """B = 65 536, N = 25, H = 256 (the wide path at the size whose GEMM kernels the benchmark runs), seeded
    synthetic weights (no H = 256 surrogate ships with the reference)."""
    p = synth_params(256, 5)
    params = {"Wih": [np.asarray(a, np.float64) for a in p["Wih"]], "Whh": [np.asarray(a, np.float64) for a in p["Whh"]],
              **{k: np.asarray(p[k], np.float64) for k in ("fcW", "fcb", "W_inp", "b_inp", "W_out")}}
    _check(*hip_and_oracle(params, 65536, 25, 24, chunk=4096), 65536, 1e-5, 1e-5, 1e-5, 1e-5)
