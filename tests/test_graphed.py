"""Captured training steps (forging-control_amd/graphed.py): a HIP-graph replay of the whole batch step
— controller training (UL/Functions.py:594-676) and surrogate training (Model_NN/Functions.py:520-569)
— must leave the parameters, losses and loss features exactly where the eager loop leaves them."""
import copy

import pytest
import torch

import forging_control_amd as fca
from forging_control_amd.graphed import CapturedStep, _make_capturable


def test_make_capturable_moves_host_step_state():
    p = torch.nn.Parameter(torch.ones(4))
    opt = torch.optim.AdamW([p], lr=1e-3)
    p.grad = torch.ones(4)
    opt.step()
    assert not opt.param_groups[0]["capturable"]
    _make_capturable(opt)
    assert opt.param_groups[0]["capturable"]
    assert opt.state[p]["step"].dtype == torch.float32 and float(opt.state[p]["step"]) == 1.0
    sgd = torch.optim.SGD([p], lr=1e-3)
    _make_capturable(sgd)   # no step state: nothing to move, nothing to refuse


def test_captured_step_refuses_host_tensors():
    p = torch.nn.Parameter(torch.ones(2))
    step = CapturedStep([p], torch.optim.SGD([p], lr=0.1), lambda x: (x.sum(),))
    with pytest.raises(RuntimeError, match="ROCm device"):
        step(torch.ones(3))


def _controller_setup(dev, seed=0):
    torch.manual_seed(seed)
    sim = fca.LSTMModel(5, 50, 4, 3).to(dev)
    for p in sim.parameters():
        p.requires_grad_(False)
    ctrl = fca.FNNModel(3, 50, 1, 1).to(dev)
    return sim, ctrl


def _controller_batches(dev, sizes, seed=1):
    g = torch.Generator(device="cpu").manual_seed(seed)
    out = []
    for B in sizes:
        X = torch.rand(B, 3, generator=g) * 2 - 1
        z = torch.rand(B, 10, 5, generator=g) * 2 - 1
        out.append((X.to(dev), torch.zeros(B, 1, device=dev), z.to(dev)))
    return out


@pytest.mark.gpu
def test_graphed_controller_training_matches_eager():
    dev = torch.device("cuda", 0)
    sim, ctrl = _controller_setup(dev)
    ctrl_g = copy.deepcopy(ctrl)
    loss_fn = fca.MPCLoss(prediction_horizon=10, alpha=20.0)
    opt = torch.optim.AdamW(ctrl.parameters(), lr=1e-3, capturable=True)
    opt_g = torch.optim.AdamW(ctrl_g.parameters(), lr=1e-3, capturable=True)
    loader = _controller_batches(dev, [15] * 6 + [7])   # the reference's B = 15, a short last batch
    step = fca.NeuralNetwork.captured_step(sim, ctrl_g, loss_fn, opt_g, dev)
    for epoch in range(3):
        l_e, f_e = fca.NeuralNetwork.train_model(loader, sim, ctrl, loss_fn, opt, dev)
        l_g, f_g = fca.NeuralNetwork.train_model(loader, sim, ctrl_g, loss_fn, opt_g, dev, step=step)
        assert abs(l_g - l_e) <= 1e-6 * max(abs(l_e), 1e-30)
        for k in ("loss", "command", "error", "prediction"):
            assert f_g[k].shape == f_e[k].shape and torch.equal(f_g[k], f_e[k]), k
        for a, b in zip(ctrl.parameters(), ctrl_g.parameters()):
            assert torch.equal(a, b)
    assert step.replays == 3 * 6 - step.warmup and step.eager_steps == step.warmup + 3


@pytest.mark.gpu
def test_graphed_controller_training_redraws_noise():
    dev = torch.device("cuda", 0)
    sim, ctrl = _controller_setup(dev)
    loss_fn = fca.MPCLoss(prediction_horizon=10, alpha=20.0)
    opt = torch.optim.AdamW(ctrl.parameters(), lr=0.0, weight_decay=0.0)   # lr 0: same weights every step
    step = fca.NeuralNetwork.captured_step(sim, ctrl, loss_fn, opt, dev, enable_noise=True)
    X, _, z = _controller_batches(dev, [64])[0]
    losses = [float(step(X, z)[0]) for _ in range(5)]
    assert step.replays == 3
    assert len(set(losses[2:])) == 3   # every replay draws fresh noise (graph-safe RNG), none is frozen


@pytest.mark.gpu
def test_graphed_surrogate_training_matches_eager():
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    m = fca.LSTMModel(5, 50, 4, 3).to(dev)
    m_g = copy.deepcopy(m)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, capturable=True)
    opt_g = torch.optim.AdamW(m_g.parameters(), lr=1e-3, capturable=True)
    g = torch.Generator(device="cpu").manual_seed(4)
    loader = [((torch.rand(B, 10, 5, generator=g) * 2 - 1).to(dev), torch.rand(B, 1, 4, generator=g).to(dev))
              for B in [256] * 5 + [100]]
    loss_fn = torch.nn.MSELoss()
    step = fca.surrogate.captured_step(m_g, loss_fn, opt_g, dev)
    for epoch in range(2):
        l_e = fca.surrogate.train_model(loader, m, loss_fn, opt, dev)
        l_g = fca.surrogate.train_model(loader, m_g, loss_fn, opt_g, dev, step=step)
        assert abs(l_g - l_e) <= 1e-6 * abs(l_e)
        for a, b in zip(m.parameters(), m_g.parameters()):
            assert torch.equal(a, b)
    assert step.replays == 2 * 5 - step.warmup


@pytest.mark.gpu
def test_graphed_step_with_grad_sync_matches_eager():
    """With a data-parallel grad_sync hook the captured step is two graphs (forward + backward, then AdamW)
    around the eager RCCL all-reduce; one rank on the box's GPU exercises that split against the eager loop."""
    import os
    import socket

    import torch.distributed as dist

    dev = torch.device("cuda", 0)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        sim, ctrl = _controller_setup(dev, seed=5)
        ctrl_g = copy.deepcopy(ctrl)
        loss_fn = fca.MPCLoss(prediction_horizon=10, alpha=20.0)
        opt = torch.optim.AdamW(ctrl.parameters(), lr=1e-3, capturable=True)
        opt_g = torch.optim.AdamW(ctrl_g.parameters(), lr=1e-3, capturable=True)
        sync = fca.distributed.GradAllReduce()
        loader = _controller_batches(dev, [32] * 5, seed=6)
        step = fca.NeuralNetwork.captured_step(sim, ctrl_g, loss_fn, opt_g, dev, grad_sync=sync)
        for _ in range(2):
            l_e, _ = fca.NeuralNetwork.train_model(loader, sim, ctrl, loss_fn, opt, dev, grad_sync=sync)
            l_g, _ = fca.NeuralNetwork.train_model(loader, sim, ctrl_g, loss_fn, opt_g, dev, grad_sync=sync, step=step)
            assert abs(l_g - l_e) <= 1e-6 * abs(l_e)
            for a, b in zip(ctrl.parameters(), ctrl_g.parameters()):
                assert torch.equal(a, b)
        assert step.replays == 2 * 5 - step.warmup and step._g_opt is not None
    finally:
        dist.destroy_process_group()
