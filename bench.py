"""Benchmark: one optimizer step of the unsupervised-MPC training path on the gfx950 rollout engine.

A step = controller(X) -> MPCLoss rollout (fused HIP forward) -> loss.backward() (fused HIP backward)
-> RCCL all-reduce of the controller gradients (N > 1 GPUs) -> AdamW, exactly the body of
NeuralNetwork.train_model (/root/reference/Unsupervised Learning/Functions.py:640-661).

Workload (BASELINE.json configs[1]): B = 65 536 trajectories per GPU, horizon N = 10, LSTM hidden 50
(3 layers, the reference's trained surrogate weights from tests/golden/weights_ref.npz), controller
3->50->1, fp32. Weak scaling: every rank runs its own 65 536 trajectories.

Prints ONE JSON line (rank 0). See DESIGN.md §Measurement for the roofline definitions.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import forging_control_amd as fca  # noqa: E402

FP32_PEAK_TFLOPS = 157.3          # MI355X dense FP32 (vector = MFMA), MI355X_MICROARCH.md
F16_PEAK_TFLOPS = 2500.0          # MI355X dense FP16/BF16 MFMA (no sparsity), MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0             # MI355X HBM3E spec
ALPHA = 20.0                      # UL/Main.py:192


def flops_per_rollout_step(H=50, L=10, layers=3, in_dim=5, ctrl_hidden=50):
    """Algorithmic FLOP of one (trajectory, horizon step): SURVEY.md §8(a3)/(d).
    Forward LSTM call: 2*[L*4H*(in+H) + (layers-1)*L*8H^2 + 4H] (readout incl.); controller 2*(3*50+50);
    backward input-gradient products: the same LSTM contraction count again (W^T . dgates)."""
    lstm = 2 * (L * 4 * H * (in_dim + H) + (layers - 1) * L * 8 * H * H + 4 * H)
    fnn = 2 * (3 * ctrl_hidden + ctrl_hidden)
    return {"fwd": lstm + fnn, "bwd": lstm + fnn, "total": 2 * (lstm + fnn)}


def hbm_bytes_per_rollout_step(N=10):
    """Compulsory HBM bytes per rollout-step: X 12 + states 200 + outputs 12 + 4N per
    trajectory, divided by N."""
    return (12 + 200 + 3 * 4 + 4 * N) / N


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/r*_pmc.json, collected by scripts/profile.sh on this workload), or None."""
    import glob
    import re
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json"))
                   if re.fullmatch(r"r\d+_pmc\.json", os.path.basename(f)))   # the rollout's, not the plant's
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    if kernel not in d:
        return None, None
    return d[kernel]["hbm_bytes_corrected"], os.path.basename(files[-1])


def load_weights(dev, H):
    if H == 50:
        w = np.load(os.path.join(ROOT, "tests", "golden", "weights_ref.npz"))
        g = lambda k: torch.as_tensor(w[k])
    else:
        gen = torch.Generator().manual_seed(0)
        shapes = {"Wih0": (4 * H, 5), "Wih1": (4 * H, H), "Wih2": (4 * H, H), "Whh0": (4 * H, H), "Whh1": (4 * H, H),
                  "Whh2": (4 * H, H), "fcW": (4, H), "fcb": (4,), "W_inp": (50, 3), "b_inp": (50,), "W_out": (1, 50)}
        rnd = {k: (torch.rand(s, generator=gen) * 2 - 1) / np.sqrt(H) for k, s in shapes.items()}
        g = lambda k: rnd[k]
    sim = fca.LSTMModel(5, H, 4, 3).to(dev)
    ctrl = fca.FNNModel(3, 50, 1, 1).to(dev)
    with torch.no_grad():
        for k in range(3):
            getattr(sim.lstm, f"weight_ih_l{k}").copy_(g(f"Wih{k}"))
            getattr(sim.lstm, f"weight_hh_l{k}").copy_(g(f"Whh{k}"))
        sim.fc.weight.copy_(g("fcW"))
        sim.fc.bias.copy_(g("fcb"))
        ctrl.fc_inp.weight.copy_(g("W_inp"))
        ctrl.fc_inp.bias.copy_(g("b_inp"))
        ctrl.fc_out.weight.copy_(g("W_out"))
    return sim, ctrl


def synth_batch(B, dev, seed):
    """SURVEY.md §8(d) input distribution (synthetic: the reference's Data/ pickle is not shipped)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    X = torch.empty(B, 3)
    X[:, 0].uniform_(-1, 1, generator=g)
    X[:, 1].uniform_(-1, 1, generator=g)
    sign = torch.randint(0, 2, (B,), generator=g).float() * 2 - 1
    X[:, 2] = sign * torch.empty(B).uniform_(0.11, 0.99, generator=g)
    S = torch.empty(B, 10, 5).uniform_(-1, 1, generator=g)
    S[:, :, 1:3].uniform_(0.0, 1.1, generator=g)
    return X.to(dev), S.to(dev)


def cpu_baseline(budget_s=15.0, B=256, N=10, threads=None):
    """The reference CPU path (stock torch ops in MPCLoss's order, oracle/rollout_torch.py) timed on the
    host: forward + backward + AdamW per step, on a bounded sample."""
    from oracle import rollout_torch as T
    threads = threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    torch.set_num_threads(threads)
    w = np.load(os.path.join(ROOT, "tests", "golden", "weights_ref.npz"))
    params = {"Wih": [w[f"Wih{k}"] for k in range(3)], "Whh": [w[f"Whh{k}"] for k in range(3)], "fcW": w["fcW"],
              "fcb": w["fcb"], "W_inp": w["W_inp"], "b_inp": w["b_inp"], "W_out": w["W_out"]}
    sim, ctrl = T.build_modules(params, torch.float32)
    opt = torch.optim.AdamW(ctrl.parameters(), lr=1e-4)
    X, S = synth_batch(B, "cpu", 99)

    def step():
        opt.zero_grad()
        u0 = ctrl(X)
        loss, _ = T.mpc_loss(sim, ctrl, X, u0, S, N, ALPHA)
        loss.backward()
        opt.step()
        return loss.item()

    step()
    t0 = time.perf_counter()
    iters = 0
    while time.perf_counter() - t0 < budget_s and iters < 200:
        step()
        iters += 1
    dt = time.perf_counter() - t0
    return {"value": B * N * iters / dt, "unit": "rollout-steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle/rollout_torch.py fwd+bwd+AdamW, B={B} N={N} H=50, {iters} steps in {dt:.1f}s, "
                      f"torch {torch.__version__}, {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=65536, help="trajectories per GPU")
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--hidden", type=int, default=50)
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--precision", choices=("fp32", "f16"), default="fp32",
                    help="fp32: reference-accurate (default, config 2); f16: config 3's reduced-precision mode")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)            # before the process group: RCCL binds each rank to its own GPU
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    B, N, H = args.batch, args.horizon, args.hidden

    sim, ctrl = load_weights(dev, H)
    if world > 1:
        fca.distributed.broadcast_params(ctrl)
    opt = torch.optim.AdamW(ctrl.parameters(), lr=1e-4)     # UL/Main.py:195
    loss_fn = fca.MPCLoss(prediction_horizon=N, alpha=ALPHA, precision=args.precision)
    sync = fca.distributed.GradAllReduce() if world > 1 else None
    X, S = synth_batch(B, dev, 1000 + rank)

    def step():
        opt.zero_grad()
        out = ctrl(X)
        loss, feats = loss_fn(sim, ctrl, X, out, S, dev)
        loss.backward()
        if sync is not None:
            sync(ctrl, B, B * world, loss)
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # per-kernel timing with events on the stream the kernels launch on (torch's current stream)
    fl = flops_per_rollout_step(H)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    fwd_ms, bwd_ms = [], []
    for _ in range(3):
        opt.zero_grad()
        out = ctrl(X)
        ev[0].record()
        loss, _ = loss_fn(sim, ctrl, X, out, S, dev)
        ev[1].record()
        ev[2].record()
        loss.backward()
        ev[3].record()
        torch.cuda.synchronize()
        fwd_ms.append(ev[0].elapsed_time(ev[1]))
        bwd_ms.append(ev[2].elapsed_time(ev[3]))
    opt.zero_grad()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = 1000.0 * dt / args.steps
    value = world * B * N / (dt / args.steps)

    if rank == 0:
        f_ms, b_ms = float(np.median(fwd_ms)), float(np.median(bwd_ms))
        dom = ("bwd", b_ms) if b_ms >= f_ms else ("fwd", f_ms)
        achieved = B * N * fl[dom[0]] / (dom[1] * 1e-3) / 1e12
        hbm_roof = HBM_PEAK_GBS * 1e9 / hbm_bytes_per_rollout_step(N)
        default_cfg = (B, N, H, args.precision) == (65536, 10, 50, "fp32")
        traffic, traffic_src = pmc_traffic(f"fcr_{dom[0]}_kernel") if default_cfg else (None, None)
        peak = FP32_PEAK_TFLOPS if args.precision == "fp32" else F16_PEAK_TFLOPS
        line = {
            "metric": "rollout-steps/s (batch x horizon), fwd+bwd+AdamW step",
            "value": value, "unit": "rollout-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32" if args.precision == "fp32" else "f16", "data": "synthetic (SURVEY §8d distribution); reference-trained LSTM/controller weights",
            "config": {"workload": f"unsupervised-MPC rollout train step, B={B}/GPU, N={N}, H={H}, 3-layer LSTM, "
                                   f"ctrl 3-50-1, {args.precision}", "batch_per_gpu": B, "global_batch": B * world, "horizon": N,
                       "hidden": H, "parallelism": f"dp{world}"},
            "roofline": {"bound": "mfma", "kernel": f"fcr_{dom[0]}_kernel", "achieved": achieved,
                         "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
                         "traffic": traffic, "traffic_unit": "bytes/launch", "traffic_source": traffic_src},
            "kernels_ms": {"fwd": f_ms, "bwd": b_ms},
            # the design's own HBM traffic (activation records and hand-off slabs, PMC-measured) against
            # 8 TB/s: how close the dominant kernel runs to the bandwidth its data movement needs
            "hbm_traffic_frac": (traffic / (dom[1] * 1e-3) / (HBM_PEAK_GBS * 1e9)) if traffic else None,
            "hbm_roofline_frac": value / world / hbm_roof,
            "loss": float(loss.item()),
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(args.cpu_budget)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
