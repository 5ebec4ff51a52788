"""GPU parity of the small-batch kernels (csrc/fcr_small.h) against the oracle and the fused kernels.

At B <= fcr_set_small_batch_limit (default 8192) the fp32 rollout of H 17..52 runs on workgroups of
four waves per 16-trajectory group (each wave owns one record quad of unit slots); above it, on the
fused one-wave-per-group kernels. Both must meet the 1e-5 bar against the fp64 oracle on every golden
case, and agree with each other to ~1e-7 (the same per-tile MFMA chains and pointwise arithmetic, up to the
compiler's fma contraction in each instance; the backward's cross-wave partial sums in another fp32 order). The two families share
the workspace layout, so a forward of one and a backward of the other also pass.
"""
import threading

import numpy as np
import pytest
import torch

import forging_control_amd as fca
from conftest import case_names, load_case, relerr
from oracle import rollout_np as R
from test_gpu_parity import DEV, FEATS, GRADS, TOL, _synth, _u0, modules, run

pytestmark = pytest.mark.gpu
native = fca._native
BIG = 1 << 30


FUSED_CASES = [n for n in case_names() if load_case(n)[0]["H"] <= 52]


def _check_oracle(o, c, name, tag):
    for k in FEATS + ("xhat",):
        assert relerr(o[k], c[f"{k}_64"]) <= TOL, (name, tag, k, relerr(o[k], c[f"{k}_64"]))
    for k, _ in GRADS:
        assert relerr(o[k], c[f"{k}_64"]) <= TOL, (name, tag, k, relerr(o[k], c[f"{k}_64"]))


@pytest.mark.parametrize("name", FUSED_CASES)
def test_small_and_fused_kernels_meet_oracle(name):
    c, params = load_case(name)
    outs = {}
    for lim in (0, BIG):
        o = run(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"], c["noise"], small_batch_limit=lim)
        # the small-batch family is built for the 8- and 13-slot tiers (H 17..52); H <= 16 stays fused
        fam = "small" if lim and c["H"] > 16 else "fused"
        assert o["families"] == (fam, fam), (name, lim, o["families"])   # both passes ran it
        _check_oracle(o, c, name, fam)
        outs[lim] = o
    for k in FEATS + ("xhat",):
        assert relerr(outs[BIG][k], outs[0][k]) <= 2e-6, (name, k, relerr(outs[BIG][k], outs[0][k]))
    for k, _ in GRADS:
        assert relerr(outs[BIG][k], outs[0][k]) <= 2e-6, (name, k, relerr(outs[BIG][k], outs[0][k]))


def _run_mixed(params, X, u0, S, N, lim_fwd, lim_bwd):
    """A forward of one family and a backward of the other: the call's options changed between the passes
    (RolloutFn carries them from the forward to its backward, so this is the only way to mix them)."""
    sim, ctrl = modules(params)
    d = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=DEV)
    u0_t = d(u0).reshape(-1, 1).requires_grad_(True)
    fn = fca.MPCLoss(prediction_horizon=N, alpha=20.0, small_batch_limit=lim_fwd)
    loss, feats = fn(sim, ctrl, d(X), u0_t, d(S), DEV)
    fn.last_call.opts.small_batch_limit = lim_bwd
    loss.backward()
    torch.cuda.synchronize()
    out = {"g_u0": u0_t.grad.reshape(-1).cpu().numpy(), "families": (fn.last_call.forward, fn.last_call.backward)}
    for k, name in GRADS[1:]:
        mod, attr = name.split(".")
        out[k] = getattr(getattr(ctrl, mod), attr).grad.cpu().numpy()
    return out


@pytest.mark.parametrize("lim_fwd,lim_bwd", [(BIG, 0), (0, BIG)])
def test_forward_of_one_family_backward_of_the_other(lim_fwd, lim_bwd):
    c, params = load_case("ref_b37_n25")
    o = _run_mixed(params, c["X"], c["u0"], c["states"], c["N"], lim_fwd, lim_bwd)
    fam = lambda lim: "small" if lim else "fused"
    assert o["families"] == (fam(lim_fwd), fam(lim_bwd)), o["families"]   # the backward ran on autograd's thread
    for k, _ in GRADS:
        assert relerr(o[k], c[f"{k}_64"]) <= TOL, (k, relerr(o[k], c[f"{k}_64"]))


@pytest.mark.parametrize("H,B,N", [(50, 1000, 3), (32, 45, 4), (40, 8, 2), (50, 1, 5)])
def test_small_kernels_ragged_and_hidden_sizes(H, B, N):
    """Many groups with a partial last one, the HS = 8 tier (two waves per group), padded units, B = 1."""
    from tests.golden.make_golden import synth_params
    params = load_case("ref_b15_n10")[1] if H == 50 else synth_params(H, 500 + H)
    X, S, _ = _synth(B, N, 600 + H + B)
    u0 = _u0(params, X)
    o = run(params, X, u0, S, N, 20.0, small_batch_limit=BIG)
    assert o["families"] == ("small", "small")
    _, f, tape = R.rollout_forward(params, X, u0, S, N, 20.0)
    g = R.rollout_backward(params, tape)
    for k in FEATS:
        assert relerr(o[k], f[k]) <= TOL, (H, B, k, relerr(o[k], f[k]))
    assert relerr(o["xhat"], f["xhat"]) <= TOL
    for k, _ in GRADS:
        assert relerr(o[k], g[k]) <= TOL, (H, B, k, relerr(o[k], g[k]))


def test_small_kernels_deterministic_and_dloss_linear():
    params = load_case("ref_b15_n10")[1]
    B, N = 300, 10
    X, S, _ = _synth(B, N, 77)
    u0 = _u0(params, X)
    a = run(params, X, u0, S, N, 20.0, small_batch_limit=BIG)
    b = run(params, X, u0, S, N, 20.0, small_batch_limit=BIG)
    c2 = run(params, X, u0, S, N, 20.0, dloss=2.0, small_batch_limit=BIG)
    for k, _ in GRADS:
        assert np.array_equal(a[k], b[k]), k
        assert np.array_equal(2.0 * a[k], c2[k]), k


def test_default_limit_routes_the_reference_batch_to_the_small_kernels():
    assert native.small_batch_limit() == 8192   # the process-wide default (tests/test_abi.py)
    c, params = load_case("ref_b15_n10")
    o = run(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"])   # options inherit the default
    assert o["families"] == ("small", "small")
    prev = native.set_small_batch_limit(0)   # a changed process default reaches calls that inherit it ...
    try:
        assert run(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"])["families"] == ("fused", "fused")
        # ... and not a call that sets its own
        o2 = run(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"], small_batch_limit=BIG)
        assert o2["families"] == ("small", "small")
    finally:
        native.set_small_batch_limit(prev)


def test_two_losses_with_different_options_run_concurrently():
    """Two MPCLoss users in one process — e.g. a training rollout beside a validation rollout — with DIFFERENT
    kernel options (small-batch kernels for one, fused for the other), each on its own thread and HIP stream at
    the same time: each gets its own kernel family in both passes (the autograd thread's backward included) and
    its own workspace, and its results are bit-identical to running it alone. No process state is changed."""
    c, params = load_case("ref_b37_n25")
    args = (params, c["X"], c["u0"], c["states"], c["N"], c["alpha"])
    alone = {lim: run(*args, small_batch_limit=lim) for lim in (0, BIG)}
    default = native.small_batch_limit()
    for rep in range(3):
        res, errs = {}, []
        barrier = threading.Barrier(2)

        def worker(lim):
            try:
                s = torch.cuda.Stream(DEV)
                with torch.cuda.stream(s):
                    barrier.wait()
                    res[lim] = run(*args, small_batch_limit=lim)
            except Exception as e:   # surfaced below
                errs.append(e)

        ts = [threading.Thread(target=worker, args=(lim,)) for lim in (0, BIG)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errs, errs
        for lim, fam in ((0, "fused"), (BIG, "small")):
            assert res[lim]["families"] == (fam, fam), (rep, lim, res[lim]["families"])
            for k in FEATS + ("xhat",) + tuple(k for k, _ in GRADS):
                assert np.array_equal(res[lim][k], alone[lim][k]), (rep, lim, k)
    assert native.small_batch_limit() == default


def test_inherited_limit_is_resolved_once_by_the_forward():
    """A call that inherits the process-wide small-batch limit runs BOTH passes with the value its forward read,
    even when the default changes before the backward (which torch may run on its autograd thread): the two
    passes never split across kernel families through process state."""
    c, params = load_case("ref_b15_n10")
    sim, ctrl = modules(params)
    d = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=DEV)
    u0_t = d(c["u0"]).reshape(-1, 1).requires_grad_(True)
    fn = fca.MPCLoss(prediction_horizon=int(c["N"]), alpha=float(c["alpha"]))   # inherits the default (8192)
    loss, _ = fn(sim, ctrl, d(c["X"]), u0_t, d(c["states"]), DEV)
    prev = native.set_small_batch_limit(0)   # "never" from here on, before the backward
    try:
        loss.backward()
        torch.cuda.synchronize()
    finally:
        native.set_small_batch_limit(prev)
    assert (fn.last_call.forward, fn.last_call.backward) == ("small", "small")
    assert fn.last_call.small_batch_limit == prev
    assert relerr(u0_t.grad.reshape(-1).cpu().numpy(), c["g_u0_64"]) <= TOL


def test_two_wide_losses_with_different_keep_budgets_run_concurrently():
    """The H > 52 path under the same concurrency as above: two MPCLoss calls at H = 64 on two
    threads and streams, one keeping every window (its backward skips the recompute) and one keeping none (its
    backward recomputes every window), at once; each is bit-identical to running it alone."""
    c, params = load_case("h64_b24_n3")
    args = (params, c["X"], c["u0"], c["states"], c["N"], c["alpha"])
    budgets = (0, 1 << 40)
    alone = {kb: run(*args, wide_keep_budget=kb) for kb in budgets}
    assert alone[0]["kept_windows"] == 0 and alone[1 << 40]["kept_windows"] == int(c["N"])
    for rep in range(3):
        res, errs = {}, []
        barrier = threading.Barrier(2)

        def worker(kb):
            try:
                s = torch.cuda.Stream(DEV)
                with torch.cuda.stream(s):
                    barrier.wait()
                    res[kb] = run(*args, wide_keep_budget=kb)
            except Exception as e:   # surfaced below
                errs.append(e)

        ts = [threading.Thread(target=worker, args=(kb,)) for kb in budgets]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errs, errs
        for kb in budgets:
            assert res[kb]["families"] == ("wide", "wide"), (rep, kb, res[kb]["families"])
            assert res[kb]["kept_windows"] == alone[kb]["kept_windows"]
            for k in FEATS + ("xhat",) + tuple(k for k, _ in GRADS):
                assert np.array_equal(res[kb][k], alone[kb][k]), (rep, kb, k)
