"""Diagnostic (round 6): the layer-pipelined small-batch kernels eager vs HIP-graph replayed, bit for bit.

    python scripts/diag_pipe_graph.py [--pipe-limit 512] [--batch 15] [--reps 20]
Prints, per replay, the largest difference of the loss features and the controller gradients against an eager run of
the same batch and weights, and whether eager runs repeat bit-identically."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import forging_control_amd as fca  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pipe-limit", type=int, default=512)
ap.add_argument("--batch", type=int, default=15)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--epochs", type=int, default=3)
ap.add_argument("--eager-pair", action="store_true", help="compare two eager training runs instead of eager vs graph")
a = ap.parse_args()
fca._native.set_small_pipe_limit(a.pipe_limit)
dev = torch.device("cuda", 0)
torch.manual_seed(0)
sim = fca.LSTMModel(5, 50, 4, 3).to(dev)
for p in sim.parameters():
    p.requires_grad_(False)
ctrl = fca.FNNModel(3, 50, 1, 1).to(dev)
loss_fn = fca.MPCLoss(prediction_horizon=10, alpha=20.0)
g = torch.Generator(device="cpu").manual_seed(1)
X = (torch.rand(a.batch, 3, generator=g) * 2 - 1).to(dev)
z = (torch.rand(a.batch, 10, 5, generator=g) * 2 - 1).to(dev)


def step():
    for p in ctrl.parameters():
        p.grad = None
    out = ctrl(X)
    loss, feats = loss_fn(sim, ctrl, X, out, z, dev)
    loss.backward()
    return [feats["loss"].detach().clone()] + [p.grad.detach().clone() for p in ctrl.parameters() if p.grad is not None]


def diff(x, y):
    return max(float((u - v).abs().max()) for u, v in zip(x, y))


ref = step()
torch.cuda.synchronize()
eager = [diff(step(), ref) for _ in range(a.reps)]
print("eager repeats: max diff", max(eager), "nonzero", sum(e > 0 for e in eager), "of", len(eager))
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        step()
torch.cuda.current_stream().wait_stream(s)
graph = torch.cuda.CUDAGraph()
static = {}
with torch.cuda.graph(graph):
    static["out"] = step()
torch.cuda.synchronize()
rep = []
for _ in range(a.reps):
    graph.replay()
    torch.cuda.synchronize()
    rep.append(diff(static["out"], ref))
print("graph replays vs eager: max diff", max(rep), "nonzero", sum(r > 0 for r in rep), "of", len(rep), rep[:8])
e2 = diff(step(), ref)
print("eager after the replays:", e2)
# the same graph replayed on OTHER inputs (copied into the captured X, z) against eager on those inputs
X0, z0 = X.clone(), z.clone()
for k in range(4):
    X.copy_((torch.rand(a.batch, 3, generator=g) * 2 - 1).to(dev))
    z.copy_((torch.rand(a.batch, 10, 5, generator=g) * 2 - 1).to(dev))
    graph.replay()
    torch.cuda.synchronize()
    got = [t.clone() for t in static["out"]]
    want = step()
    torch.cuda.synchronize()
    print(f"new inputs {k}: graph vs eager max diff {diff(got, want):.3e}")
X.copy_(X0)
z.copy_(z0)

# the controller training loop of tests/test_graphed.py: eager train_model against the captured step, per epoch
sys.path.insert(0, os.path.join(ROOT, "tests"))
import copy  # noqa: E402
from test_graphed import _controller_batches, _controller_setup  # noqa: E402

sim, ctrl = _controller_setup(dev)
ctrl_g = copy.deepcopy(ctrl)
ctrl_0 = copy.deepcopy(ctrl)   # the one-workgroup kernels (pipe limit 0), eager: the arbiter
opt_0 = torch.optim.AdamW(ctrl_0.parameters(), lr=1e-3, capturable=True)
opt = torch.optim.AdamW(ctrl.parameters(), lr=1e-3, capturable=True)
opt_g = torch.optim.AdamW(ctrl_g.parameters(), lr=1e-3, capturable=True)
loader = _controller_batches(dev, [15] * 6 + [7])
cstep = None if a.eager_pair else fca.NeuralNetwork.captured_step(sim, ctrl_g, loss_fn, opt_g, dev)
bad = 0
for epoch in range(a.epochs):
    l_e, f_e = fca.NeuralNetwork.train_model(loader, sim, ctrl, loss_fn, opt, dev)
    l_g, f_g = fca.NeuralNetwork.train_model(loader, sim, ctrl_g, loss_fn, opt_g, dev, step=cstep)
    prev = fca._native.set_small_pipe_limit(0)
    l_0, f_0 = fca.NeuralNetwork.train_model(loader, sim, ctrl_0, loss_fn, opt_0, dev)
    fca._native.set_small_pipe_limit(prev)
    for name, f in (("eager-pipe", f_e), ("second", f_g)):
        d = max(float((f[k] - f_0[k]).abs().max()) for k in ("loss", "command", "error", "prediction"))
        print(f"epoch {epoch} {name} vs one-workgroup eager: max feature diff {d:.3e}")
    for k in ("loss", "command", "error", "prediction"):
        d = (f_g[k] - f_e[k]).abs()
        idx = torch.nonzero(d).flatten().tolist()
        if idx:
            print(f"epoch {epoch} {k}: max diff {float(d.max()):.3e} at {idx[:12]} of {d.numel()}")
    pd = max(float((p - q).detach().abs().max()) for p, q in zip(ctrl.parameters(), ctrl_g.parameters()))
    if pd > 0:
        bad += 1
        print(f"epoch {epoch}: loss {l_e} vs {l_g}; parameter max diff {pd:.3e} -> resynchronised")
        with torch.no_grad():
            for p, q, r in zip(ctrl.parameters(), ctrl_g.parameters(), ctrl_0.parameters()):
                q.copy_(p)
                r.copy_(p)
print(f"epochs with a difference: {bad} of {a.epochs}")
