"""GPU parity of the layer-pipelined small-batch kernels (csrc/fcr_pipe.h).

At B <= fcr_set_small_pipe_limit (default 512, at most 32 groups of 16 trajectories) the small-batch family runs one
workgroup per LSTM layer and group, handing cells between the layer workgroups through the sequence slabs and
progress counters; with the limit at 0 the same batches run on one workgroup per group (csrc/fcr_small.h). Both
geometries run the same per-cell arithmetic (fwd16_cell, sb_step) and must meet the 1e-5 bar against the fp64 oracle;
against each other they agree to the compiler's fma contraction in each instance (measured bit-identical in
profiles/round6_b15_pipe_*). They share the workspace layout, so a forward of one and a backward of the other pass.
"""
import numpy as np
import pytest
import torch

import forging_control_amd as fca
from conftest import load_case, relerr
from oracle import rollout_np as R
from test_gpu_parity import DEV, FEATS, GRADS, TOL, _synth, _u0, modules, run

pytestmark = pytest.mark.gpu
native = fca._native
BIG = 1 << 30


def _oracle(params, X, u0, S, N):
    _, f, tape = R.rollout_forward(params, X, u0, S, N, 20.0)
    return f, R.rollout_backward(params, tape)


def _with_pipe_limit(lim, fn):
    prev = native.set_small_pipe_limit(lim)
    try:
        return fn()
    finally:
        native.set_small_pipe_limit(prev)


@pytest.mark.parametrize("H,B,N", [(50, 15, 10), (50, 1, 5), (32, 45, 4), (50, 256, 10), (50, 512, 3), (40, 37, 25),
                                   (50, 7, 1), (50, 16, 2), (50, 17, 2), (24, 100, 3)])
def test_layer_pipelined_small_kernels_meet_oracle_and_match_one_workgroup(H, B, N):
    from tests.golden.make_golden import synth_params
    params = load_case("ref_b15_n10")[1] if H == 50 else synth_params(H, 700 + H)
    X, S, _ = _synth(B, N, 800 + H + B)
    u0 = _u0(params, X)
    assert native.small_pipe_limit() == 512
    pipe = run(params, X, u0, S, N, 20.0, small_batch_limit=BIG)
    one = _with_pipe_limit(0, lambda: run(params, X, u0, S, N, 20.0, small_batch_limit=BIG))
    assert pipe["families"] == ("small", "small") and one["families"] == ("small", "small")
    f, g = _oracle(params, X, u0, S, N)
    for k in FEATS + ("xhat",):
        ref = f[k]
        assert relerr(pipe[k], ref) <= TOL, (H, B, N, k, relerr(pipe[k], ref))
        assert relerr(pipe[k], one[k]) <= 1e-6, (H, B, N, k, relerr(pipe[k], one[k]))
    for k, _ in GRADS:
        assert relerr(pipe[k], g[k]) <= TOL, (H, B, N, k, relerr(pipe[k], g[k]))
        assert relerr(pipe[k], one[k]) <= 1e-6, (H, B, N, k, relerr(pipe[k], one[k]))


def _with_pipe_sets(sets, fn):
    prev = native.set_small_pipe_sets(sets)
    try:
        return fn()
    finally:
        native.set_small_pipe_sets(prev)


@pytest.mark.parametrize("H,B,N", [(50, 15, 10), (50, 40, 25), (32, 17, 2), (50, 9, 1), (50, 3, 4)])
def test_window_sets_meet_oracle_and_agree(H, B, N):
    """S = 1 .. 4 window sets (forward 2 S, backward 3 S workgroups per group, the backward at most 3 sets; set s takes
    windows s, s + S, ...): the same cells, the cost sums in window order, so the same bits for every S; and the fp64
    oracle at 1e-5."""
    from tests.golden.make_golden import synth_params
    params = load_case("ref_b15_n10")[1] if H == 50 else synth_params(H, 900 + H)
    X, S, _ = _synth(B, N, 1000 + H + B + N)
    u0 = _u0(params, X)
    assert native.small_pipe_sets() == 0
    outs = {k: _with_pipe_sets(k, lambda: run(params, X, u0, S, N, 20.0, small_batch_limit=BIG)) for k in (1, 2, 3, 4)}
    f, g = _oracle(params, X, u0, S, N)
    for k in FEATS + ("xhat",):
        assert relerr(outs[3][k], f[k]) <= TOL, (H, B, N, k, relerr(outs[3][k], f[k]))
    for k, _ in GRADS:
        assert relerr(outs[3][k], g[k]) <= TOL, (H, B, N, k, relerr(outs[3][k], g[k]))
    for sets in (2, 3, 4):
        for k in FEATS + ("xhat",) + tuple(k for k, _ in GRADS):
            assert np.array_equal(outs[sets][k], outs[1][k]), (sets, H, B, N, k, relerr(outs[sets][k], outs[1][k]))


def test_layer_pipelined_golden_reference_batch():
    """The reference's own batch (B = 15, N = 10, its trained weights) against the committed fp64 fixture."""
    c, params = load_case("ref_b15_n10")
    o = run(params, c["X"], c["u0"], c["states"], c["N"], c["alpha"], c["noise"])
    assert o["families"] == ("small", "small")
    for k in FEATS + ("xhat",):
        assert relerr(o[k], c[f"{k}_64"]) <= TOL, (k, relerr(o[k], c[f"{k}_64"]))
    for k, _ in GRADS:
        assert relerr(o[k], c[f"{k}_64"]) <= TOL, (k, relerr(o[k], c[f"{k}_64"]))


@pytest.mark.parametrize("fwd_lim,bwd_lim", [(512, 0), (0, 512)])
def test_pipelined_and_one_workgroup_passes_mix(fwd_lim, bwd_lim):
    """A forward of one geometry and the backward of the other (the process-wide limit changed between them)."""
    c, params = load_case("ref_b37_n25")
    sim, ctrl = modules(params)
    d = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=DEV)
    u0_t = d(c["u0"]).reshape(-1, 1).requires_grad_(True)
    prev = native.set_small_pipe_limit(fwd_lim)
    try:
        fn = fca.MPCLoss(prediction_horizon=c["N"], alpha=20.0, small_batch_limit=BIG)
        loss, _ = fn(sim, ctrl, d(c["X"]), u0_t, d(c["states"]), DEV)
        torch.cuda.synchronize()
        native.set_small_pipe_limit(bwd_lim)
        loss.backward()
        torch.cuda.synchronize()
    finally:
        native.set_small_pipe_limit(prev)
    out = {"g_u0": u0_t.grad.reshape(-1).cpu().numpy()}
    for k, name in GRADS[1:]:
        mod, attr = name.split(".")
        out[k] = getattr(getattr(ctrl, mod), attr).grad.cpu().numpy()
    for k, _ in GRADS:
        assert relerr(out[k], c[f"{k}_64"]) <= TOL, (k, relerr(out[k], c[f"{k}_64"]))


def test_layer_pipelined_deterministic():
    params = load_case("ref_b15_n10")[1]
    X, S, _ = _synth(200, 10, 91)
    u0 = _u0(params, X)
    a = run(params, X, u0, S, 10, 20.0, small_batch_limit=BIG)
    b = run(params, X, u0, S, 10, 20.0, small_batch_limit=BIG)
    for k in FEATS + ("xhat",) + tuple(k for k, _ in GRADS):
        assert np.array_equal(a[k], b[k]), k


def test_layer_pipelined_graph_replay_on_new_inputs():
    """A captured step replayed on inputs other than the capture's must match eager on those inputs: the progress
    counters are cleared by a kernel node each replay (a captured hipMemsetAsync left them stale — the layer-0
    workgroup then read the previous replay's hand-off rows; profiles/round6_b15_pipe_graph.log)."""
    torch.manual_seed(0)
    sim = fca.LSTMModel(5, 50, 4, 3).to(DEV)
    for p in sim.parameters():
        p.requires_grad_(False)
    ctrl = fca.FNNModel(3, 50, 1, 1).to(DEV)
    loss_fn = fca.MPCLoss(prediction_horizon=10, alpha=20.0)
    g = torch.Generator(device="cpu").manual_seed(5)
    draw = lambda: ((torch.rand(15, 3, generator=g) * 2 - 1).to(DEV), (torch.rand(15, 10, 5, generator=g) * 2 - 1).to(DEV))
    X, z = draw()

    def step():
        for p in ctrl.parameters():
            p.grad = None
        loss, feats = loss_fn(sim, ctrl, X, ctrl(X), z, DEV)
        loss.backward()
        return [feats["loss"].detach().clone()] + [p.grad.detach().clone() for p in ctrl.parameters() if p.grad is not None]

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = step()
    for _ in range(3):
        Xn, zn = draw()
        X.copy_(Xn)
        z.copy_(zn)
        graph.replay()
        got = [t.clone() for t in out]
        want = step()
        torch.cuda.synchronize()
        for a, b in zip(got, want):
            assert torch.equal(a, b)


def _rollout_node(loss):
    node, seen = loss.grad_fn, []
    while node is not None and not hasattr(node, "ws"):
        seen.extend(f for f, _ in node.next_functions if f is not None)
        node = seen.pop(0) if seen else None
    assert node is not None
    return node


def test_layer_pipelined_second_backward_of_one_forward():
    """Two fcr_backward calls on one forward's workspace (as the C ABI allows): the second starts from counters the
    first left zeroed (its last workgroup resets them), so the accumulated gradients are exactly twice the first.
    Through autograd a second backward is refused (the first releases the workspace); the test hands it back."""
    c, params = load_case("ref_b15_n10")
    sim, ctrl = modules(params)
    d = lambda v: torch.as_tensor(np.asarray(v, np.float32), device=DEV)
    fn = fca.MPCLoss(prediction_horizon=c["N"], alpha=20.0, small_batch_limit=BIG)
    u0 = ctrl(d(c["X"]))
    loss, _ = fn(sim, ctrl, d(c["X"]), u0, d(c["states"]), DEV)
    node = _rollout_node(loss)
    ws = node.ws
    loss.backward(retain_graph=True)
    params_g = [p for p in ctrl.parameters() if p.grad is not None]
    assert params_g
    first = [p.grad.clone() for p in params_g]
    with pytest.raises(RuntimeError, match="second time"):
        loss.backward(retain_graph=True)
    node.ws = ws
    loss.backward()
    torch.cuda.synchronize()
    for g1, p in zip(first, params_g):
        assert torch.isfinite(g1).all()
        assert torch.equal(p.grad, 2 * g1)


def test_pipelined_random_sweep_matches_one_workgroup():
    """A seeded sweep over (H, B, N) — every window-set count the host picks, ragged groups, N from 1 to 25 — against
    the one-workgroup kernels (1e-6, as above) with every output finite: the hand-off protocol under many shapes."""
    from tests.golden.make_golden import synth_params
    rng = np.random.default_rng(2026)
    for case in range(16):
        H = int(rng.choice([24, 32, 40, 50]))
        B = int(rng.integers(1, 513))
        N = int(rng.integers(1, 26))
        params = synth_params(H, 1200 + case)
        X, S, _ = _synth(B, N, 1300 + case)
        u0 = _u0(params, X)
        pipe = run(params, X, u0, S, N, 20.0, small_batch_limit=BIG)
        one = _with_pipe_limit(0, lambda: run(params, X, u0, S, N, 20.0, small_batch_limit=BIG))
        for k in FEATS + ("xhat",) + tuple(k for k, _ in GRADS):
            assert np.isfinite(pipe[k]).all(), (case, H, B, N, k)
            assert relerr(pipe[k], one[k]) <= 1e-6, (case, H, B, N, k, relerr(pipe[k], one[k]))
