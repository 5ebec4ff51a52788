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
# A band trajectory's g_u0 may differ from the fp64 value at u0 by a flip — but then it IS the fp64 derivative on the
# other side of that kink: the one-sided derivative at u0 +- d for a small shift d (oracle.rollout_torch.one_sided_g_u0).
# Every band trajectory above 1e-5 must match one of those within 1e-5 (the flip stated, not tolerated), and flips
# may be no more frequent than in stock torch fp32 on the same batch (max(10, 2x its count)). Stock torch fp32's own
# band error is reported beside HIP's.


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


def _inputs(B, N, seed):
    """The batch of a test: ("own", seed) synth_inputs (tests/golden/make_golden.py); ("bench", seed) the benchmark's
    own batch (bench.py synth_batch, rank 0's seed 1000), so the bench line's check and this test see the same data."""
    kind, k = seed
    if kind == "bench":
        import bench
        return bench.synth_batch(B, DEV, k)
    X, S, _ = synth_inputs(B, N, k)
    d = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=DEV)
    return d(X), d(S)


MAX_FLIPS_EXAMINED = 64   # one-sided derivatives are one fp64 rollout each: beyond this many the count check fails anyway


def kink_band(params, got, ref, ref32, Xd, Sd, u0, N, examine=True):
    """The band's g_u0 error of the HIP path and of stock torch fp32 (both against the fp64 values), each one's count of
    band trajectories above 1e-5, and (examine: the fp32-accurate mode) for HIP's: whether each one's g_u0 is a
    one-sided fp64 derivative at its kink."""
    B = Xd.shape[0]
    band = ~(T.kink_margin(params, Xd.double(), ref["xhat"].reshape(B, N, 4)) > DELTA)
    den = ref["g_u0"].abs().max()
    e_all = (got["g_u0"].double() - ref["g_u0"]).abs() / den
    e = e_all[band]
    e32 = (ref32["g_u0"].double() - ref["g_u0"]).abs()[band] / den
    hip, t32 = (float(e.max()), float(e32.max())) if e.numel() else (0.0, 0.0)
    flagged = torch.nonzero(band & (e_all > 1e-5)).reshape(-1).tolist()
    side = (T.one_sided_g_u0(params, Xd, u0, Sd, N, 20.0, flagged, B, device=DEV)
            if examine and len(flagged) <= MAX_FLIPS_EXAMINED else {})
    explained = {}
    for r in (flagged if side else []):
        g = float(got["g_u0"][r])
        best = min(side[r], key=lambda sg: abs(g - sg[1]))
        explained[r] = {"err_at_u0": float(e_all[r]), "shift": best[0], "err_one_sided": abs(g - best[1]) / float(den)}
    return {"kink_trajectories": int(band.sum()), "g_u0_err_in_kink_band": hip, "torch_fp32_err_in_kink_band": t32,
            "kink_above_1e-5": len(flagged), "torch_fp32_kink_above_1e-5": int((e32 > 1e-5).sum()),
            "flips": explained}, ~band


def hip_and_oracle(params, B, N, seed, precision="fp32", chunk=16384):
    """Returns (err, info). err: per-trajectory outputs over ALL trajectories, g_u0 outside the kink band, the
    full-batch parameter gradients and the loss (each max|hip - ref| / max|ref| over the batch); info: the kink
    band (kink_band) and stock torch fp32's own errors on the same batch."""
    Xd, Sd = _inputs(B, N, seed)
    got, u0 = _hip(params, Xd, Sd, N, precision)
    ref = T.loss_and_grads_chunked(params, Xd, u0, Sd, N, 20.0, device=DEV, chunk=chunk)
    ref32 = T.loss_and_grads_chunked(params, Xd, u0, Sd, N, 20.0, device=DEV, chunk=chunk, dtype=torch.float32)
    info, reg = kink_band(params, got, ref, ref32, Xd, Sd, u0, N, examine=precision == "fp32")
    err = {k: _err(got[k], ref[k]) for k in FEATS + PARAMS}
    err["g_u0"] = _err(got["g_u0"], ref["g_u0"], reg)
    err["loss_scalar"] = _err(got["loss_scalar"], ref["loss_scalar"])
    info["torch_fp32"] = {k: _err(ref32[k], ref[k]) for k in PARAMS + ("xhat",)}
    info["torch_fp32"]["g_u0"] = _err(ref32["g_u0"], ref["g_u0"], reg)
    print(seed, {k: f"{v:.2e}" for k, v in err.items()}, info)
    return err, info


def _check(err, info, B, tol_traj, tol_gu0, tol_grad, tol_loss, kink=True):
    assert err["loss_scalar"] <= tol_loss, err
    assert max(err[k] for k in FEATS) <= tol_traj, err          # every trajectory, no exclusion
    assert err["g_u0"] <= tol_gu0, err                           # outside the kink band
    assert max(err[k] for k in PARAMS) <= tol_grad, err          # full-batch sums, flips included
    if kink:   # the band: every g_u0 above 1e-5 is the fp64 one-sided derivative of its kink; flips no more frequent
        # than stock torch fp32's on the same batch
        assert info["kink_above_1e-5"] <= max(10, 2 * info["torch_fp32_kink_above_1e-5"]), info
        assert len(info["flips"]) == info["kink_above_1e-5"], info   # every one examined ...
        for r, f in info["flips"].items():                            # ... and a one-sided derivative
            assert f["err_one_sided"] <= 1e-5, (r, f, info)
    else:      # reduced precision: the band is held to the mode's own g_u0 tolerance
        assert info["g_u0_err_in_kink_band"] <= tol_gu0, info


@pytest.fixture(scope="module")
def ref_params():
    return load_case("ref_b15_n10")[1]


BENCH = ("bench", 1000)   # bench.py's batch (rank 0)


@pytest.mark.parametrize("seed", [("own", 21), BENCH])
def test_config2_full_batch_parameter_gradients(ref_params, seed):
    """B = 65 536, N = 10, H = 50, fp32: every output and the controller gradients summed over 655 360 terms."""
    _check(*hip_and_oracle(ref_params, 65536, 10, seed), 65536, 1e-5, 1e-5, 1e-5, 1e-5)


@pytest.mark.parametrize("seed", [("own", 22), BENCH])
def test_config3_full_batch_fp32(ref_params, seed):
    """B = 262 144 in the default fp32-accurate mode (on the bench seed: the batch whose committed line showed a
    1.9e-3 band error, round 3 — held here to stock torch fp32's own band error on the same batch)."""
    _check(*hip_and_oracle(ref_params, 262144, 10, seed), 262144, 1e-5, 1e-5, 1e-5, 1e-5)


@pytest.mark.parametrize("seed", [("own", 23), BENCH])
def test_config3_full_batch_f16(ref_params, seed):
    """B = 262 144 in config 3's reduced-precision mode (f16 gate products in both passes, fp32 accumulate) at the
    stated tolerances (tests/test_gpu_precision.py)."""
    from test_gpu_precision import TOL_FEATS, TOL_GRADS_F16_FULL, TOL_GU0_F16_FULL, TOL_LOSS
    _check(*hip_and_oracle(ref_params, 262144, 10, seed, precision="f16"), 262144, TOL_FEATS, TOL_GU0_F16_FULL,
           TOL_GRADS_F16_FULL, TOL_LOSS, kink=False)   # the f16 forward's own error exceeds the kink bar


def _params_of(sim, ctrl):
    cpu = lambda t: t.detach().double().cpu().numpy()
    return {"Wih": [cpu(getattr(sim.lstm, f"weight_ih_l{k}")) for k in range(3)],
            "Whh": [cpu(getattr(sim.lstm, f"weight_hh_l{k}")) for k in range(3)], "fcW": cpu(sim.fc.weight),
            "fcb": cpu(sim.fc.bias), "W_inp": cpu(ctrl.fc_inp.weight), "b_inp": cpu(ctrl.fc_inp.bias),
            "W_out": cpu(ctrl.fc_out.weight)}


@pytest.mark.parametrize("seed", [("own", 24), BENCH])
def test_config5_full_batch(seed):
    """B = 65 536, N = 25, H = 256 (the wide path at the size whose GEMM kernels the benchmark runs), seeded
    synthetic weights (no H = 256 surrogate ships with the reference): the test's own, or the benchmark's weights
    and batch."""
    if seed[0] == "bench":
        import bench
        params = _params_of(*bench.load_weights(DEV, 256))
    else:
        p = synth_params(256, 5)
        params = {"Wih": [np.asarray(a, np.float64) for a in p["Wih"]], "Whh": [np.asarray(a, np.float64) for a in p["Whh"]],
                  **{k: np.asarray(p[k], np.float64) for k in ("fcW", "fcb", "W_inp", "b_inp", "W_out")}}
    _check(*hip_and_oracle(params, 65536, 25, seed, chunk=4096), 65536, 1e-5, 1e-5, 1e-5, 1e-5)


@pytest.mark.parametrize("B", [32768, 32767])
def test_wide_backward_geometries_at_their_batch_threshold(B):
    """The wide backward's layers >= 1 run 256 x 256-trajectory workgroups from B = 32 768 on and 256 x 128 below
    (fcr_abi.hip launch_fb): both sides of the threshold at H = 264 (Hp = 320: three 256-column blocks, three row-bound
    slots) and N = 2, every trajectory against the fp64 oracle."""
    p = synth_params(264, 7)
    params = {"Wih": [np.asarray(a, np.float64) for a in p["Wih"]], "Whh": [np.asarray(a, np.float64) for a in p["Whh"]],
              **{k: np.asarray(p[k], np.float64) for k in ("fcW", "fcb", "W_inp", "b_inp", "W_out")}}
    _check(*hip_and_oracle(params, B, 2, ("own", 26), chunk=8192), B, 1e-5, 1e-5, 1e-5, 1e-5)
