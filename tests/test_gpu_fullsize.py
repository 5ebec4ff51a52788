"""Full-size parity at the benchmarked batch sizes (BASELINE.json configs 2, 3 and 5): the gfx950 rollout's
loss, per-trajectory features and x̂ of EVERY trajectory, per-trajectory u0 gradients AND the
controller-parameter gradients — sums over all B·N (trajectory, step) terms — against the stock-torch restatement (oracle/rollout_torch.py)
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
FEATS = ("loss", "command", "error", "prediction", "xhat")
PARAMS = ("g_W_inp", "g_b_inp", "g_W_out")
# kink band: trajectories whose fp64 rollout passes within DELTA of a ReLU / Hardtanh / constraint kink
# (oracle.rollout_torch.kink_margin), where an fp32 mask can flip against fp64's: one term's SLOPE changes by O(1),
# so only d loss / d u0 of that trajectory can move — every forward output is continuous across the kink and is
# compared over ALL trajectories, and the parameter gradients are the full-batch sums, flips included.
DELTA = 1e-5
# a flipped mask swaps one of a trajectory's ~N (50 + 4) piecewise slopes; the kink-band g_u0 error must stay far
# below O(1) of the batch's largest gradient (the worst seen: 1.9e-4) and be the exception, not the rule
KINK_GU0_MAX = 1e-3
KINK_GU0_FRAC = 1e-3   # at most this share of the batch may exceed the 1e-5 bar (flips), of B


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
    den = r.abs().max()
    if rows is not None:
        a, r = a[rows], r[rows]
    return float((a - r).abs().max() / den) if a.numel() else 0.0


def hip_and_oracle(params, B, N, seed, precision="fp32", chunk=16384):
    """Returns (err, info). err: per-trajectory outputs over ALL trajectories, g_u0 outside the kink band, the
    full-batch parameter gradients and the loss (each max|hip - ref| / max|ref| over the batch); info: the kink
    band's size, its largest g_u0 error and how many of its trajectories exceed 1e-5."""
    X, S, _ = synth_inputs(B, N, seed)
    d = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=DEV)
    Xd, Sd = d(X), d(S)
    got, u0 = _hip(params, Xd, Sd, N, precision)
    ref = T.loss_and_grads_chunked(params, Xd, u0, Sd, N, 20.0, device=DEV, chunk=chunk)
    reg = T.kink_margin(params, Xd.double(), ref["xhat"].reshape(B, N, 4)) > DELTA
    err = {k: _err(got[k], ref[k]) for k in FEATS + PARAMS}
    err["g_u0"] = _err(got["g_u0"], ref["g_u0"], reg)
    err["loss_scalar"] = _err(got["loss_scalar"], ref["loss_scalar"])
    band = ~reg
    e_band = (got["g_u0"].double() - ref["g_u0"]).abs()[band] / ref["g_u0"].abs().max()
    info = {"kink_trajectories": int(band.sum()),
            "g_u0_err_in_kink_band": float(e_band.max()) if e_band.numel() else 0.0,
            "kink_above_1e-5": int((e_band > 1e-5).sum())}
    print({k: f"{v:.2e}" for k, v in err.items()}, info)
    return err, info


def _check(err, info, B, tol_traj, tol_gu0, tol_grad, tol_loss, kink=True):
    assert err["loss_scalar"] <= tol_loss, err
    assert max(err[k] for k in FEATS) <= tol_traj, err          # every trajectory, no exclusion
    assert err["g_u0"] <= tol_gu0, err                           # outside the kink band
    assert max(err[k] for k in PARAMS) <= tol_grad, err          # full-batch sums, flips included
    if kink:   # the kink band's g_u0: bounded, and flips the exception
        assert info["g_u0_err_in_kink_band"] <= KINK_GU0_MAX, info
        assert info["kink_above_1e-5"] <= KINK_GU0_FRAC * B, info
    else:      # reduced precision: the band is held to the mode's own g_u0 tolerance
        assert info["g_u0_err_in_kink_band"] <= tol_gu0, info


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
           TOL_GRADS_F16FWD_FULL, TOL_LOSS, kink=False)   # the f16 forward's own error exceeds the kink bar


def test_config5_full_batch():
    """B = 65 536, N = 25, H = 256 (the wide path at the size whose GEMM kernels the benchmark runs), seeded
    synthetic weights (no H = 256 surrogate ships with the reference)."""
    p = synth_params(256, 5)
    params = {"Wih": [np.asarray(a, np.float64) for a in p["Wih"]], "Whh": [np.asarray(a, np.float64) for a in p["Whh"]],
              **{k: np.asarray(p[k], np.float64) for k in ("fcW", "fcb", "W_inp", "b_inp", "W_out")}}
    _check(*hip_and_oracle(params, 65536, 25, 24, chunk=4096), 65536, 1e-5, 1e-5, 1e-5, 1e-5)
