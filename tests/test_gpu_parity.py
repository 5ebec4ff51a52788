"""GPU parity: the gfx950 rollout (through the C ABI) against the oracle fixtures.

Metric: per tensor max|hip - ref| / max|ref| <= 1e-5 (north_star's fp32 bar), against
both the fp64 NumPy oracle and the stock-torch fp32 restatement. Full-size (B = 65 536) cases are
checked through size-independent properties: sampled per-trajectory parity, determinism, shard
independence, exact dloss linearity.
"""
import numpy as np
import pytest
import torch

import forging_control_amd as fca
from conftest import load_case, relerr
from oracle import rollout_np as R

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = "cuda:0"
FEATS = ("loss", "command", "error", "prediction")
GRADS = (("g_u0", None), ("g_W_inp", "fc_inp.weight"), ("g_b_inp", "fc_inp.bias"), ("g_W_out", "fc_out.weight"))


def modules(params, dev=DEV):
    H = params["Whh"][0].shape[1]
    sim = fca.LSTMModel(5, H, 4, 3).to(dev)
    ctrl = fca.FNNModel(3, params["W_inp"].shape[0], 1, 1).to(dev)
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
    for p in sim.parameters():
        p.requires_grad_(True)      # as in the reference: frozen by the optimizer, not by autograd
    return sim, ctrl


def run(params, X, u0, states, N, alpha, noise=None, dloss=1.0, **loss_kw):
    """One MPCLoss forward + backward on the GPU; loss_kw: its per-call kernel options (small_batch_limit,
    wide_keep_budget). out["families"] = the kernel family (forward, backward) the call launched."""
    sim, ctrl = modules(params)
    d = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=DEV)
    u0_t = d(u0).reshape(-1, 1).requires_grad_(True)
    fn = fca.MPCLoss(prediction_horizon=N, alpha=alpha, **loss_kw)
    loss, feats = fn(sim, ctrl, d(X), u0_t, d(states), DEV, enable_noise=noise is not None,
                     noise=None if noise is None else d(noise))
    (loss * dloss).backward()
    torch.cuda.synchronize()
    out = {k: v.detach().cpu().numpy() for k, v in feats.items()}
    out["loss_scalar"] = loss.item()
    out["xhat"] = fn.last_trajectory.cpu().numpy()
    out["g_u0"] = u0_t.grad.reshape(-1).cpu().numpy()
    for k, name in GRADS[1:]:
        mod, attr = name.split(".")
        out[k] = getattr(getattr(ctrl, mod), attr).grad.cpu().numpy()
    out["lstm_grad_untouched"] = all(p.grad is None for p in sim.parameters())
    out["families"] = (fn.last_call.forward, fn.last_call.backward)
    out["kept_windows"] = fn.last_call.kept_windows
    return out


def test_golden_case_parity(golden):
    name, c, params = golden
    o = run(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"], c["noise"])
    assert abs(o["loss_scalar"] - float(c["loss64"])) <= TOL * abs(float(c["loss64"]))
    for k in FEATS + ("xhat",):
        assert relerr(o[k], c[f"{k}_64"]) <= TOL, (name, k, relerr(o[k], c[f"{k}_64"]))
        assert relerr(o[k], c[f"{k}_32"]) <= TOL, (name, k, "vs torch fp32")
    for k, _ in GRADS:
        assert relerr(o[k], c[f"{k}_64"]) <= TOL, (name, k, relerr(o[k], c[f"{k}_64"]))
        assert relerr(o[k], c[f"{k}_32"]) <= TOL, (name, k, "vs torch fp32")
    assert o["lstm_grad_untouched"]   # documented deviation: LSTM weight grads are not produced


def _synth(B, N, seed, wide=False):
    from tests.golden.make_golden import synth_inputs
    return synth_inputs(B, N, seed, wide)


@pytest.fixture(scope="module")
def ref_params():
    return load_case("ref_b15_n10")[1]


def _u0(params, X):
    u, _ = R.fnn_forward(np.asarray(X, np.float64), params["W_inp"], params["b_inp"], params["W_out"])
    return u.astype(np.float32)


def test_full_size_sampled_parity(ref_params):
    """B = 65 536, N = 10, H = 50 (BASELINE config 2): 48 random trajectories re-run on the fp64 oracle."""
    B, N = 65536, 10
    X, S, _ = _synth(B, N, 11)
    u0 = _u0(ref_params, X)
    o = run(ref_params, X, u0, S, N, 20.0)
    idx = np.random.default_rng(0).choice(B, 48, replace=False)
    _, f, tape = R.rollout_forward(ref_params, X[idx], u0[idx], S[idx], N, 20.0)
    g = R.rollout_backward(ref_params, tape)
    for k in ("loss", "command", "error"):
        assert relerr(o[k][idx], f[k]) <= TOL, k
    pred = o["prediction"].reshape(B, N)[idx].reshape(-1)
    assert relerr(pred, f["prediction"]) <= TOL
    assert relerr(o["xhat"][idx], f["xhat"]) <= TOL
    # per-trajectory u0 gradient carries the 1/B of the batch mean
    assert relerr(o["g_u0"][idx] * B, g["g_u0"] * len(idx)) <= TOL
    assert np.isfinite(o["loss_scalar"]) and abs(o["loss_scalar"] - o["loss"].mean()) <= 1e-6 * abs(o["loss_scalar"])


def test_param_grads_at_2048(ref_params):
    B, N = 2048, 10
    X, S, _ = _synth(B, N, 12, wide=True)
    u0 = _u0(ref_params, X)
    o = run(ref_params, X, u0, S, N, 20.0)
    _, f, tape = R.rollout_forward(ref_params, X, u0, S, N, 20.0)
    g = R.rollout_backward(ref_params, tape)
    for k, _ in GRADS:
        assert relerr(o[k], g[k]) <= TOL, (k, relerr(o[k], g[k]))
    assert relerr(o["loss"], f["loss"]) <= TOL


def test_deterministic_and_dloss_linear(ref_params):
    B, N = 4096, 10
    X, S, _ = _synth(B, N, 13)
    u0 = _u0(ref_params, X)
    a = run(ref_params, X, u0, S, N, 20.0)
    b = run(ref_params, X, u0, S, N, 20.0)
    c2 = run(ref_params, X, u0, S, N, 20.0, dloss=2.0)
    for k in FEATS + ("xhat",):
        assert np.array_equal(a[k], b[k]), k
    for k, _ in GRADS:
        assert np.array_equal(a[k], b[k]), k              # fixed-order reductions: bit-reproducible
        assert np.array_equal(2.0 * a[k], c2[k]), k       # exact linearity in the incoming gradient


def test_shard_independence(ref_params):
    """Trajectories never interact before the batch mean: a 16-aligned shard reproduces its rows."""
    B, N = 96, 10
    X, S, _ = _synth(B, N, 14)
    u0 = _u0(ref_params, X)
    full = run(ref_params, X, u0, S, N, 20.0)
    part = run(ref_params, X[32:64], u0[32:64], S[32:64], N, 20.0)
    for k in ("loss", "command", "error"):
        assert np.array_equal(full[k][32:64], part[k]), k
    assert np.array_equal(full["xhat"][32:64], part["xhat"])
    # the gradients carry 1/B: B=96 vs 32 is not a power-of-two rescaling, so the split-f16 operands of
    # the backward products round differently (fcr_f16.h) — equal to ~1e-6, not bit-equal
    assert relerr(full["g_u0"][32:64] * B, part["g_u0"] * 32) <= 4e-6


@pytest.mark.parametrize("B", [1, 17, 1000])
def test_ragged_batches(ref_params, B):
    N = 3
    X, S, _ = _synth(B, N, 15 + B)
    u0 = _u0(ref_params, X)
    o = run(ref_params, X, u0, S, N, 20.0)
    _, f, tape = R.rollout_forward(ref_params, X, u0, S, N, 20.0)
    g = R.rollout_backward(ref_params, tape)
    assert relerr(o["prediction"], f["prediction"]) <= TOL
    assert relerr(o["loss"], f["loss"]) <= TOL
    for k, _ in GRADS:
        assert relerr(o[k], g[k]) <= TOL, k


def test_enable_noise_draws_reference_stream(ref_params):
    """enable_noise draws randn_like(x0)*0.01 once per horizon step in order (Functions.py:1401,1439)."""
    B, N = 40, 5
    X, S, _ = _synth(B, N, 16)
    u0 = _u0(ref_params, X)
    sim, ctrl = modules(ref_params)
    d = lambda a: torch.as_tensor(a, device=DEV)
    fn = fca.MPCLoss(N, 20.0)
    torch.manual_seed(123)
    l1, f1 = fn(sim, ctrl, d(X), d(u0).reshape(-1, 1), d(S), DEV, enable_noise=True)
    torch.manual_seed(123)
    nz = torch.stack([torch.randn(B, 4, device=DEV) * 0.01 for _ in range(N)], dim=1)
    l2, f2 = fn(sim, ctrl, d(X), d(u0).reshape(-1, 1), d(S), DEV, noise=nz, enable_noise=True)
    assert torch.equal(f1["loss"], f2["loss"]) and torch.equal(f1["prediction"], f2["prediction"])


def test_train_step_integration(ref_params):
    """controller(X) -> MPCLoss -> backward -> AdamW, as train_model does (Functions.py:640-658): the
    u0 gradient flows back into the caller's controller graph and adds to the in-loss gradients."""
    c, params = load_case("ref_b256_n10")
    sim, ctrl = modules(params)
    d = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=DEV)
    opt = torch.optim.AdamW(ctrl.parameters(), lr=1e-4)
    opt.zero_grad()
    X = d(c["X"])
    out = ctrl(X)
    loss, _ = fca.MPCLoss(c["N"], c["alpha"])(sim, ctrl, X, out, d(c["states"]), DEV)
    loss.backward()
    # expected: in-loss grads (golden) + J_u0^T g_u0 through the fp64 controller
    Wi = torch.tensor(params["W_inp"], requires_grad=True)
    bi = torch.tensor(params["b_inp"], requires_grad=True)
    Wo = torch.tensor(params["W_out"], requires_grad=True)
    Xd = torch.tensor(np.asarray(c["X"], np.float64))
    u = torch.nn.functional.hardtanh(torch.relu(Xd @ Wi.T + bi) @ Wo.T).reshape(-1)
    u.backward(torch.tensor(c["g_u0_64"]))
    exp = {"fc_inp.weight": Wi.grad.numpy() + c["g_W_inp_64"], "fc_inp.bias": bi.grad.numpy() + c["g_b_inp_64"],
           "fc_out.weight": Wo.grad.numpy() + c["g_W_out_64"]}
    for name, e in exp.items():
        mod, attr = name.split(".")
        got = getattr(getattr(ctrl, mod), attr).grad.cpu().numpy()
        assert relerr(got, e) <= TOL, name
    before = {n: p.detach().clone() for n, p in ctrl.named_parameters()}
    opt.step()
    for n, p in ctrl.named_parameters():
        if p.grad is None:
            assert torch.equal(p, before[n])      # fc_int: no grad -> skipped by AdamW
    assert ctrl.fc_int.weight.grad is None


def test_bad_shapes_raise(ref_params):
    sim, ctrl = modules(ref_params)
    X = torch.zeros(8, 3, device=DEV)
    with pytest.raises(ValueError):
        fca.MPCLoss(10, 20.0)(sim, ctrl, X, ctrl(X), torch.zeros(8, 9, 5, device=DEV), DEV)


@pytest.mark.parametrize("H,B,N", [(40, 48, 4), (7, 33, 3), (21, 17, 2), (52, 20, 3)])
def test_any_hidden_size_up_to_52(H, B, N):
    """A hidden size between the built tiers (16, 32, 52 units) runs with zero padding units; checked
    against the fp64 oracle on seeded synthetic weights (parity unpinned: no reference output)."""
    from tests.golden.make_golden import synth_params
    params = synth_params(H, 100 + H)
    X, S, _ = _synth(B, N, 200 + H)
    u0 = _u0(params, X)
    o = run(params, X, u0, S, N, 20.0)
    _, f, tape = R.rollout_forward(params, X, u0, S, N, 20.0)
    g = R.rollout_backward(params, tape)
    for k in FEATS:
        assert relerr(o[k], f[k]) <= TOL, (H, k, relerr(o[k], f[k]))
    assert relerr(o["xhat"], f["xhat"]) <= TOL
    for k, _ in GRADS:
        assert relerr(o[k], g[k]) <= TOL, (H, k, relerr(o[k], g[k]))


@pytest.mark.parametrize("dloss", [1e-4, 1e4])
def test_wide_path_any_incoming_gradient_scale(dloss):
    """H > 52 (config 5's path, split-f16 products): the dgates enter the f16 operands scaled by each trajectory row's
    own power of two (fcr_wbwd.h), so a scaled loss (loss * dloss).backward() neither underflows nor overflows them."""
    c, params = load_case("h64_b24_n3")
    o = run(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"], c["noise"], dloss=dloss)
    for k, _ in GRADS:
        assert relerr(o[k] / dloss, c[f"{k}_64"]) <= TOL, (k, relerr(o[k] / dloss, c[f"{k}_64"]))


@pytest.mark.parametrize("H,B,N", [(54, 300, 3), (57, 77, 2), (96, 520, 4), (64, 129, 2), (128, 300, 3), (192, 260, 2),
                                   (200, 140, 2), (264, 130, 2)])
def test_wide_path_hidden_sizes(H, B, N):
    """H > 52 at sizes the golden cases do not hit. Every H runs the hand-written cells (round 5: no rocBLAS on the
    rollout) at H padded to whole 64-unit blocks with zero-weight units: H = 54, 57 (10 and 7 padding units, the odd
    H), 200 (56) and 264 (56: Hp = 320, so the fused backward cell's [input gradient | dh_{t-1}] product spans three
    column blocks of 256 and its row bounds three slots), beside the unpadded 64, 96 (padded to 128), 128 and 192 (two
    column blocks with the dh columns straddling them); ragged last blocks of 128 trajectories. Against the fp64
    oracle on seeded synthetic weights (parity unpinned: no reference output at these sizes)."""
    from tests.golden.make_golden import synth_params
    params = synth_params(H, 300 + H)
    X, S, _ = _synth(B, N, 400 + H)
    u0 = _u0(params, X)
    o = run(params, X, u0, S, N, 20.0)
    _, f, tape = R.rollout_forward(params, X, u0, S, N, 20.0)
    g = R.rollout_backward(params, tape)
    for k in FEATS:
        assert relerr(o[k], f[k]) <= TOL, (H, k, relerr(o[k], f[k]))
    assert relerr(o["xhat"], f["xhat"]) <= TOL
    for k, _ in GRADS:
        assert relerr(o[k], g[k]) <= TOL, (H, k, relerr(o[k], g[k]))


def test_wide_path_kept_windows_equal_recompute():
    """H > 52: windows whose cell state the forward keeps (MPCLoss(wide_keep_budget=...), fcr_options) skip the
    backward's recompute; the kept pre-activations and c are the recompute's, so every output and gradient is the
    same bit for bit with none, one or all windows kept, and all match the fp64 oracle. The budget is the call's
    own: the process-wide default is left untouched."""
    from tests.golden.make_golden import synth_params
    H, B, N = 64, 200, 4
    params = synth_params(H, 364)
    X, S, _ = _synth(B, N, 464)
    u0 = _u0(params, X)
    default = fca._native.wide_keep_budget()
    outs = []
    per_window = 4 * 3 * 10 * B * 5 * H   # bytes of one kept window
    # none; smaller than one window (none); all windows; exactly one window (the last)
    for budget, kept in ((0, 0), (1, 0), (1 << 40, N), (per_window + 4096, 1)):
        o = run(params, X, u0, S, N, 20.0, wide_keep_budget=budget)
        assert o["kept_windows"] == kept and o["families"] == ("wide", "wide"), (budget, o["kept_windows"])
        outs.append(o)
    assert fca._native.wide_keep_budget() == default
    for o in outs[1:]:
        for k in FEATS + ("xhat",) + tuple(k for k, _ in GRADS):
            assert np.array_equal(o[k], outs[0][k]), k
    _, f, tape = R.rollout_forward(params, X, u0, S, N, 20.0)
    g = R.rollout_backward(params, tape)
    for k, _ in GRADS:
        assert relerr(outs[2][k], g[k]) <= TOL, (k, relerr(outs[2][k], g[k]))


@pytest.mark.parametrize("case", ["ref_b15_n10", "h64_b24_n3"])
def test_nonfinite_incoming_gradient_propagates(case):
    """A non-finite upstream gradient (an overflowed loss scale) must come out non-finite, as torch's does —
    not as partly-zeroed finite gradients that hide the overflow from GradScaler / anomaly detection — on the
    fused path (H <= 52) and the wide path (H > 52, whose per-row dgate scales see the non-finite bound)."""
    c, params = load_case(case)
    o = run(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"], c["noise"], dloss=float("inf"))
    for k, _ in GRADS:
        assert not np.isfinite(o[k]).all(), k


@pytest.mark.parametrize("H", [50, 64])
@pytest.mark.parametrize("scale", [1e5, 3e7])
def test_unscaled_window_values_stay_finite_like_torch_fp32(H, scale):
    """Window values beyond the f16 range (states x 1e5; x 3e7 ~ unscaled press pressures in Pa,
    results/*_dataframe.txt) would overflow the f16 split of the gate-product operands (hi = f16(v) = inf ->
    NaN), where torch fp32 stays finite. The range guard (fcr_pack.h) runs those columns on v 2^-s_c against
    W_ih0 2^s_c: the rollout stays finite and close to fp64 on the fused path and the GEMM path. At these
    magnitudes a layer-0 gate pre-activation carries an absolute error ~|W||v| 2^-24 in fp32 (torch) and
    ~|W||v| 2^-22 in the split product (the dropped lo·lo term): the rare gate whose |W||v| ~ 1e7 terms cancel
    to near 0 lands on a different sigmoid value in any fp32 implementation. Bound: 5e-5, or 4x torch fp32's
    own distance to fp64 (measured at x 3e7, H = 50: prediction 1.3e-5 vs torch fp32 1.3e-7)."""
    from oracle import rollout_torch as TT
    from tests.golden.make_golden import synth_params
    params = load_case("ref_b15_n10")[1] if H == 50 else synth_params(H, 7)
    if H != 50:
        params = {"Wih": [np.asarray(a, np.float64) for a in params["Wih"]],
                  "Whh": [np.asarray(a, np.float64) for a in params["Whh"]],
                  **{k: np.asarray(params[k], np.float64) for k in ("fcW", "fcb", "W_inp", "b_inp", "W_out")}}
    B, N = 48, 4
    X, S, _ = _synth(B, N, 31)
    S = (S * scale).astype(np.float32)
    u0 = _u0(params, X)
    o = run(params, X, u0, S, N, 20.0)
    r64 = TT.loss_and_grads(params, X, u0, S, N, 20.0, dtype=torch.float64)
    r32 = TT.loss_and_grads(params, X, u0, S, N, 20.0, dtype=torch.float32)
    for k in FEATS + ("xhat",) + tuple(g for g, _ in GRADS):
        assert np.isfinite(o[k]).all(), k
        e_hip, e_t32 = relerr(o[k], r64[k]), relerr(r32[k], r64[k])
        assert e_hip <= max(5e-5, 4 * e_t32), (k, e_hip, e_t32)


def test_wide_forget_dgates_near_their_f16_margin():
    """H > 52 backward: the per-row dgate scale 2^(13 - e) bounds every scaled dgate by |dc_t| times a local derivative
    <= 1, except the forget row, dc_t c_{t-1} f (1 - f), which relies on |c_{t-1}| <= t from each window's zero
    initial state (Functions.py:349-350; fcr_wide.h kWideDgExp). This drives that row toward its margin: input and
    cell gates saturated (i = g = 1) and the forget gate at 1 for eight steps, so c grows by one per step, then at
    f = 1/2 (its largest f (1 - f)) in the window's ninth row: c_{t-1} f (1 - f) = 2 where the bound allows 9/4, i.e.
    scaled forget dgates ~16 k of f16's 65 504. The gradients must still meet the fp64 oracle."""
    from tests.golden.make_golden import synth_params
    H, B, N = 64, 48, 2
    p = synth_params(H, 4242)
    X, S, _ = _synth(B, N, 4243)
    wih0 = p["Wih"][0].copy()
    wih0[0:H, 3] += 30.0            # input gate <- column 3 (z)
    wih0[2 * H:3 * H, 3] += 30.0    # cell gate  <- column 3
    wih0[H:2 * H, 0] += 30.0        # forget gate <- column 0 (y_dot)
    p["Wih"][0] = wih0.astype(np.float32).astype(np.float64)
    S[:, :, 3] = 1.0
    S[:, :8, 0] = 1.0               # f = 1 over rows 0..7
    S[:, 8:, 0] = 0.0               # f ~ 1/2 from row 8 (the other weights add O(0.1) to the pre-activation)
    u0 = _u0(p, X)
    o = run(p, X, u0, S, N, 20.0)
    assert o["families"] == ("wide", "wide")
    _, f, tape = R.rollout_forward(p, X, u0, S, N, 20.0)
    g = R.rollout_backward(p, tape)
    assert np.all(np.isfinite(o["xhat"]))
    for k in FEATS + ("xhat",):
        assert relerr(o[k], f[k]) <= TOL, (k, relerr(o[k], f[k]))
    for k, _ in GRADS:
        assert np.all(np.isfinite(o[k])), k
        assert relerr(o[k], g[k]) <= TOL, (k, relerr(o[k], g[k]))
