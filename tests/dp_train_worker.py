"""World-size-N data-parallel training through the package's launcher (test helper, CPU / gloo).

``python tests/dp_train_worker.py --ranks N --out DIR`` re-launches itself as N ranks with
``forging_control_amd.launch.spawn_ranks`` — the launcher ``bench.py --gpus N`` uses — and each rank runs
the real ``NeuralNetwork.train_model(..., grad_sync=GradAllReduce())`` over its contiguous shard of every
global batch (the reference's B = 15, so shards are uneven: 8 / 7, and the last batch of 7 splits 4 / 3; at
8 ranks the last batch leaves rank 7 an EMPTY shard). The loss is the package's own ``MPCLoss`` on the CPU
(its reference op sequence, functions.py) over the reference's trained surrogate — the GPU kernels are not
needed to test the data-parallel plumbing. Every rank writes its final controller parameters and epoch
losses to DIR.
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import forging_control_amd as fca  # noqa: E402

N_HORIZON, ALPHA = 3, 20.0
BATCHES = [15, 15, 7]


def surrogate():
    w = np.load(os.path.join(ROOT, "tests", "golden", "weights_ref.npz"))
    sim = fca.LSTMModel(5, 50, 4, 3)
    with torch.no_grad():
        for k in range(3):
            getattr(sim.lstm, f"weight_ih_l{k}").copy_(torch.as_tensor(w[f"Wih{k}"]))
            getattr(sim.lstm, f"weight_hh_l{k}").copy_(torch.as_tensor(w[f"Whh{k}"]))
        sim.fc.weight.copy_(torch.as_tensor(w["fcW"]))
        sim.fc.bias.copy_(torch.as_tensor(w["fcb"]))
    return sim


def global_batches(seed=0):
    g = torch.Generator().manual_seed(seed)
    out = []
    for b in BATCHES:
        X = torch.rand(b, 3, generator=g) * 2 - 1
        z = torch.rand(b, 10, 5, generator=g) * 2 - 1
        z[:, :, 1:3] = torch.rand(b, 10, 2, generator=g) * 1.1
        out.append((X, torch.zeros(b, 1), z))
    return out


class EagerCapturedStep(fca.graphed.CapturedStep):
    """The captured-step path of train_model (``step=``: _train_model_captured, CapturedStep.skip_empty) with the
    graph replay replaced by the same step run eagerly, so it runs on the CPU under gloo (the graphs themselves are
    covered on the GPU by tests/test_graphed.py)."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        for group in self.optimizer.param_groups:   # no graph here: AdamW keeps its host-side step (CPU params)
            group["capturable"] = False

    def __call__(self, *batch):
        if batch[0].shape[0] == 0:   # as on the device, where the rollout refuses B = 0 (fcr_forward check_dims)
            raise RuntimeError("CapturedStep called on an empty shard")
        out = self._eager(batch)
        return tuple(t.detach() for t in out)


def train(loader, grad_sync=None, epochs=2, captured=False):
    torch.manual_seed(11)
    ctrl = fca.FNNModel(3, 50, 1, 1)
    if grad_sync is not None:
        fca.distributed.broadcast_params(ctrl)
    opt = torch.optim.AdamW(ctrl.parameters(), lr=1e-2)
    sim = surrogate()
    loss_fn = fca.MPCLoss(N_HORIZON, ALPHA)
    step = None
    if captured:
        def body(X, z):
            loss, f = loss_fn(sim, ctrl, X, ctrl(X), z, "cpu")
            loss.backward()
            return (loss.detach(), f["loss"], f["command"], f["error"], f["prediction"])
        sync = (lambda X, z: grad_sync(ctrl, X.shape[0])) if grad_sync is not None else None
        step = EagerCapturedStep(ctrl.parameters(), opt, body, sync)
    losses = [fca.NeuralNetwork.train_model(loader, sim, ctrl, loss_fn, opt, "cpu", grad_sync=grad_sync,
                                            step=step)[0]
              for _ in range(epochs)]
    return torch.cat([p.detach().reshape(-1) for p in ctrl.parameters()]).numpy(), np.array(losses)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--out", required=True)
    ap.add_argument("--captured", action="store_true", help="train through the captured-step path (step=...)")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ:
        sys.exit(fca.launch.spawn_ranks(args.ranks, os.path.abspath(__file__), sys.argv[1:], timeout=300))
    rank, _, world = fca.launch.rank_env()
    assert world == args.ranks
    dist.init_process_group("gloo")
    shard = []
    for X, y, z in global_batches():
        lo, hi = fca.distributed.shard_range(X.shape[0], rank, world)
        shard.append((X[lo:hi], y[lo:hi], z[lo:hi]))
    params, losses = train(shard, fca.distributed.GradAllReduce(), captured=args.captured)
    np.savez(os.path.join(args.out, f"rank{rank}.npz"), params=params, losses=losses, world=dist.get_world_size())
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
