"""Eager vs HIP-graph-replayed training steps (forging-control_amd/graphed.py), one JSON line per case.

controller: the UL training step (controller(X) -> MPCLoss rollout -> backward -> AdamW,
UL/Functions.py:640-658) at the reference's batch B = 15 (UL/Main.py) and larger batches.
surrogate: the Model_NN step (LSTMModel forward, MSE, backward, AdamW; Model_NN/Functions.py:541-566) at
the reference's B = 256. Both loops take the batch from device tensors, as the drop-in's loaders do.
The eager arm reads the loss per step (``loss.item()``, as the reference's loop does) only in the
"sync" variant; both timed arms are otherwise asynchronous so launch cost, not the host round trip, is
what they compare.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import forging_control_amd as fca  # noqa: E402


def timed(fn, steps, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return 1000.0 * (time.perf_counter() - t0) / steps


def controller_case(B, steps, dev):
    sim, ctrl = bench.load_weights(dev, 50)
    X, S = bench.synth_batch(B, dev, 7)
    loss_fn = fca.MPCLoss(prediction_horizon=10, alpha=bench.ALPHA)
    opt = torch.optim.AdamW(ctrl.parameters(), lr=1e-4, capturable=True)

    def eager():
        opt.zero_grad()
        loss, _ = loss_fn(sim, ctrl, X, ctrl(X), S, dev)
        loss.backward()
        opt.step()
        return loss

    def eager_sync():
        return float(eager().item())

    step = fca.NeuralNetwork.captured_step(sim, ctrl, loss_fn, opt, dev)
    graphed = lambda: step(X, S)
    res = {"eager": timed(eager, steps), "eager_item": timed(eager_sync, steps), "graphed": timed(graphed, steps)}
    assert step.replays > 0
    return res


def surrogate_case(B, steps, dev):
    torch.manual_seed(0)
    m = fca.LSTMModel(5, 50, 4, 3).to(dev)
    X = torch.rand(B, 10, 5, device=dev) * 2 - 1
    Y = torch.rand(B, 1, 4, device=dev)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, capturable=True)
    mse = torch.nn.MSELoss()

    def eager():
        opt.zero_grad()
        loss = mse(m(X, dev), Y.squeeze())
        loss.backward()
        opt.step()
        return loss

    def eager_sync():
        return float(eager().item())

    step = fca.surrogate.captured_step(m, mse, opt, dev)
    graphed = lambda: step(X, Y)
    res = {"eager": timed(eager, steps), "eager_item": timed(eager_sync, steps), "graphed": timed(graphed, steps)}
    assert step.replays > 0
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--controller-B", type=int, nargs="*", default=[15, 256, 4096, 65536])
    ap.add_argument("--surrogate-B", type=int, nargs="*", default=[256, 4096])
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for name, Bs, fn, unit_per in (("controller", args.controller_B, controller_case, 10),
                                   ("surrogate", args.surrogate_B, surrogate_case, 1)):
        for B in Bs:
            steps = args.steps if B <= 4096 else 10
            r = fn(B, steps, dev)
            print(json.dumps({"workload": f"{name} training step", "B": B, "ms_per_step": r,
                              "units_per_s_graphed": B * unit_per / (r["graphed"] * 1e-3),
                              "unit": "rollout-steps/s" if name == "controller" else "windows/s",
                              "speedup_vs_eager": r["eager"] / r["graphed"],
                              "speedup_vs_eager_item": r["eager_item"] / r["graphed"]}), flush=True)


if __name__ == "__main__":
    main()
