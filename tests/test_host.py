"""CPU: host-side mirror of the reference interface and the data-parallel plumbing."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import forging_control_amd as fca
from conftest import GOLDEN


def test_reference_state_dicts_load_into_mirror_modules():
    w = np.load(os.path.join(GOLDEN, "weights_ref.npz"))
    sim = fca.LSTMModel(5, 50, 4, 3)
    sd = {f"lstm.weight_ih_l{k}": torch.tensor(w[f"Wih{k}"]) for k in range(3)}
    sd.update({f"lstm.weight_hh_l{k}": torch.tensor(w[f"Whh{k}"]) for k in range(3)})
    sd.update({"fc.weight": torch.tensor(w["fcW"]), "fc.bias": torch.tensor(w["fcb"])})
    sim.load_state_dict(sd)          # strict: same keys as UL/Model_NN/results/model_NN.pt
    ctrl = fca.FNNModel(3, 50, 1, 1, torch.nn.ReLU, bias=True)
    keys = set(ctrl.state_dict())
    assert keys == {"fc_inp.weight", "fc_inp.bias", "fc_int.weight", "fc_int.bias", "fc_out.weight"}


def test_fnn_forward_matches_oracle():
    from oracle import rollout_np as R
    torch.manual_seed(0)
    ctrl = fca.FNNModel(3, 50, 1, 1)
    x = torch.randn(64, 3, dtype=torch.float64) * 3
    ctrl = ctrl.double()
    u_np, _ = R.fnn_forward(x.numpy(), ctrl.fc_inp.weight.detach().numpy(), ctrl.fc_inp.bias.detach().numpy(),
                            ctrl.fc_out.weight.detach().numpy())
    assert np.allclose(ctrl(x).detach().numpy()[:, 0], u_np, atol=1e-14)


def _cpu_modules(params):
    H = params["Whh"][0].shape[1]
    sim = fca.LSTMModel(5, H, 4, 3)
    ctrl = fca.FNNModel(3, params["W_inp"].shape[0], 1, 1)
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
    return sim, ctrl


def test_mpcloss_cpu_device_matches_fixture(golden):
    """MPCLoss with device = cpu (the reference's no-GPU branch, UL/Main.py:38): the package's host path
    (functions.MPCLoss._forward_host — the reference's op sequence on the caller's modules, not the oracle)
    against the committed fp64 fixture at the 1e-5 bar: loss, loss features, x̂, d loss/d u0 and the
    controller-parameter gradients after loss.backward()."""
    from conftest import relerr
    name, c, params = golden
    sim, ctrl = _cpu_modules(params)
    f32 = lambda a: torch.as_tensor(np.asarray(a, np.float32))
    X, S = f32(c["X"]), f32(c["states"])
    u0 = f32(c["u0"]).reshape(-1, 1).requires_grad_(True)
    fn = fca.MPCLoss(prediction_horizon=c["N"], alpha=c["alpha"])
    noise = None if c["noise"] is None else f32(c["noise"])
    loss, f = fn(sim, ctrl, X, u0, S, "cpu", enable_noise=noise is not None, noise=noise)
    loss.backward()
    got = {k: v.detach().numpy() for k, v in f.items()}
    got["xhat"] = fn.last_trajectory.numpy()
    got["g_u0"] = u0.grad.reshape(-1).numpy()
    g = lambda p: (p.grad if p.grad is not None else torch.zeros_like(p)).numpy()   # N = 1: no in-loss controller call
    got["g_W_inp"], got["g_b_inp"], got["g_W_out"] = g(ctrl.fc_inp.weight), g(ctrl.fc_inp.bias), g(ctrl.fc_out.weight)
    assert abs(loss.item() - float(c["loss64"])) <= 1e-5 * abs(float(c["loss64"]))
    for k in ("loss", "command", "error", "prediction", "xhat", "g_u0", "g_W_inp", "g_b_inp", "g_W_out"):
        assert relerr(got[k], c[f"{k}_64"]) <= 1e-5, (name, k, relerr(got[k], c[f"{k}_64"]))
    # the reference's autograd also reaches the frozen LSTM's weights (never stepped, UL/Main.py:195)
    assert all(p.grad is not None for p in sim.lstm.parameters())


def test_mpcloss_cpu_noise_draws_in_reference_order():
    """enable_noise on the CPU draws randn_like(x̂) * 0.01 after every surrogate call (Functions.py:1401, 1439):
    with the generator reseeded, the same draws as a pre-drawn (B, N, 4) noise tensor taken in that order."""
    from conftest import load_case
    c, params = load_case("ref_b15_n10")
    sim, ctrl = _cpu_modules(params)
    X, S = torch.as_tensor(c["X"]), torch.as_tensor(c["states"])
    u0 = torch.as_tensor(c["u0"]).reshape(-1, 1)
    fn = fca.MPCLoss(prediction_horizon=c["N"], alpha=20.0)
    torch.manual_seed(5)
    l1, f1 = fn(sim, ctrl, X, u0, S, "cpu", enable_noise=True)
    torch.manual_seed(5)
    noise = torch.stack([torch.randn(X.shape[0], 4) * 0.01 for _ in range(c["N"])], dim=1)
    l2, f2 = fn(sim, ctrl, X, u0, S, "cpu", enable_noise=True, noise=noise)
    assert torch.equal(l1, l2) and torch.equal(f1["prediction"], f2["prediction"])
    l3, _ = fn(sim, ctrl, X, u0, S, "cpu")
    assert not torch.equal(l1, l3)


def test_rollout_entry_refuses_cpu_tensors():
    """The functional kernel entry (rollout.rollout) runs on the ROCm device or raises: no hidden fallback."""
    sim = fca.LSTMModel(5, 50, 4, 3)
    ctrl = fca.FNNModel(3, 50, 1, 1)
    X = torch.zeros(4, 3)
    with pytest.raises(RuntimeError, match="ROCm device only"):
        fca.rollout.rollout(X, ctrl(X), torch.zeros(4, 10, 5), fca.functions._controller_params(ctrl),
                            fca.functions._simulator_params(sim), 10, 20.0)


def test_mpcloss_rejects_unsupported_models():
    sim = fca.LSTMModel(5, 50, 4, 3, bias=True)
    ctrl = fca.FNNModel(3, 50, 1, 1)
    with pytest.raises(NotImplementedError):
        fca.functions._simulator_params(sim)
    with pytest.raises(NotImplementedError):
        fca.functions._controller_params(fca.FNNModel(3, 50, 1, 2))


def test_shard_range_partitions_batch():
    for B, W in [(65536, 8), (15, 4), (7, 8)]:
        spans = [fca.distributed.shard_range(B, r, W) for r in range(W)]
        assert spans[0][0] == 0 and spans[-1][1] == B
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def _dp_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = fca.FNNModel(3, 50, 1, 1)
    B_global = 12
    lo, hi = fca.distributed.shard_range(B_global, rank, world)
    g = torch.Generator().manual_seed(1)
    X = torch.randn(B_global, 3, generator=g)
    # local mean loss over the shard; the all-reduced grad must equal the global-mean grad
    loss = model(X[lo:hi]).pow(2).mean()
    loss.backward()
    red_loss = fca.distributed.GradAllReduce()(model, hi - lo, B_global, loss)
    out[rank] = (torch.cat([p.grad.reshape(-1) for p in model.parameters() if p.grad is not None]).numpy(),
                 float(red_loss))
    dist.destroy_process_group()


def test_grad_allreduce_equals_global_mean_gloo_world2():
    port = 29500 + os.getpid() % 1000
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_dp_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    torch.manual_seed(0)
    model = fca.FNNModel(3, 50, 1, 1)
    X = torch.randn(12, 3, generator=torch.Generator().manual_seed(1))
    loss = model(X).pow(2).mean()
    loss.backward()
    ref = torch.cat([p.grad.reshape(-1) for p in model.parameters() if p.grad is not None]).numpy()
    for r in (0, 1):
        assert np.allclose(res[r][0], ref, atol=1e-6)
        assert abs(res[r][1] - loss.item()) < 1e-6


def _dp_adamw_worker(rank, world, port, out):
    """Three optimizer steps exactly as bench.py / train_model(grad_sync=...) run them per rank."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(rank + 7)                       # ranks start from different weights ...
    model = fca.FNNModel(3, 50, 1, 1)
    fca.distributed.broadcast_params(model)           # ... until rank 0's are broadcast
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
    sync = fca.distributed.GradAllReduce()
    B_global = 10
    lo, hi = fca.distributed.shard_range(B_global, rank, world)
    for step in range(3):
        X = torch.randn(B_global, 3, generator=torch.Generator().manual_seed(100 + step))
        opt.zero_grad()
        loss = (model(X[lo:hi]) - 0.3).pow(2).mean()
        loss.backward()
        sync(model, hi - lo, B_global, loss)
        opt.step()
    out[rank] = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).numpy()
    dist.destroy_process_group()


def test_dp_adamw_steps_equal_full_batch_gloo_world3():
    """World size 3 with ragged shards (4/3/3): after three AdamW steps every rank holds the parameters
    of one process training on the whole batch (the reduction order differs, hence allclose)."""
    port = 30500 + os.getpid() % 1000
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_dp_adamw_worker, args=(3, port, out), nprocs=3, join=True)
        res = dict(out)
    torch.manual_seed(0 + 7)
    model = fca.FNNModel(3, 50, 1, 1)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
    for step in range(3):
        X = torch.randn(10, 3, generator=torch.Generator().manual_seed(100 + step))
        opt.zero_grad()
        (model(X) - 0.3).pow(2).mean().backward()
        opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).numpy()
    for r in range(3):
        assert np.allclose(res[r], ref, atol=1e-6), r
    assert np.array_equal(res[0], res[1]) and np.array_equal(res[1], res[2])


def test_inference_refuses_cpu_tensors():
    """No CPU fallback: the product path needs the ROCm device (the oracle is test infrastructure)."""
    import pytest
    import torch
    import forging_control_amd as fca
    sim = fca.LSTMModel(5, 50, 4, 3)
    with pytest.raises(RuntimeError, match="ROCm device"):
        fca.simulate_step(sim, torch.zeros(2, 10, 5))


@pytest.mark.parametrize("ranks,captured", [(2, False), (8, False), (8, True)])
def test_train_model_data_parallel_through_launcher_gloo(tmp_path, ranks, captured):
    """The launcher bench.py --gpus N uses (forging_control_amd.launch) starts N gloo ranks that each run the
    real NeuralNetwork.train_model(grad_sync=GradAllReduce()) with the package's MPCLoss (CPU path) on UNEVEN
    shards of the reference's B = 15 batches (2 ranks: 8/7, last batch 4/3; 8 ranks: 2/2/.../1, and the last
    batch of 7 leaves rank 7 an EMPTY shard, which must still join the all-reduce): after two epochs every rank
    holds bit-identical parameters equal to one process training on the whole batches. captured: the same through
    train_model's captured-step path (step=..., graph replay stood in by the eager step on the CPU), whose empty
    shard must join the all-reduce too (CapturedStep.skip_empty)."""
    import subprocess
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    import dp_train_worker as W
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dp_train_worker.py")
    rc = subprocess.run([sys.executable, script, "--ranks", str(ranks), "--out", str(tmp_path)] +
                        (["--captured"] if captured else []), timeout=400).returncode
    assert rc == 0
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(ranks)]
    assert all(int(r["world"]) == ranks for r in res)
    assert all(np.array_equal(res[0]["params"], r["params"]) for r in res[1:])
    ref_params, _ = W.train(W.global_batches())
    assert np.allclose(res[0]["params"], ref_params, rtol=0, atol=2e-6), np.abs(res[0]["params"] - ref_params).max()
    assert not np.allclose(ref_params, W.train(W.global_batches(), epochs=0)[0])   # training moved them
