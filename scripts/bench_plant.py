"""Benchmark of the batched forging-press plant, one JSON line.

Workload: B trajectories x S steps of F = Ruge_Kuta(TS = 1 ms, M = 4) over forging_model
(Functions.py:1615-1781), fp64, states and commands resident in HBM. A unit is one trajectory-step
(4 RK4 stages = 16 right-hand sides). CPU baseline: the fp64 NumPy restatement (oracle/plant_np.py,
vectorised over the batch, one thread) on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import forging_control_amd as fca  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1 << 20)
    ap.add_argument("--S", type=int, default=50)
    ap.add_argument("--substeps", type=int, default=4)
    ap.add_argument("--smooth", type=int, default=0)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    B, S = args.B, args.S
    base = torch.tensor([0.04, 0.3, 1.0e7, 5.0e6, 0.1], dtype=torch.float64)
    x0 = (base * (1 + 0.5 * torch.rand(B, 5, generator=g, dtype=torch.float64))).to(dev)
    u = (0.3 * (torch.rand(B, S, generator=g, dtype=torch.float64) - 0.3)).to(dev)
    F = fca.ForgingRK4(1e-3, args.substeps, bool(args.smooth))
    for _ in range(2):
        F.rollout(x0, u)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(args.iters):
        out = F.rollout(x0, u)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / args.iters
    assert torch.isfinite(out).all()
    units = B * S
    line = {"metric": "plant trajectory-steps/s", "value": units / (ms * 1e-3), "unit": "trajectory-steps/s",
            "ms_per_launch": ms, "dtype": "f64",
            "config": {"workload": "forging_model RK4 (TS=1ms, M=%d%s)" % (args.substeps, ", smooth" if args.smooth else ""),
                       "B": B, "S": S},
            "hbm_bytes_per_unit": 48.0, "hbm_gbs": units * 48.0 / (ms * 1e-3) / 1e9}
    # CPU baseline: the NumPy restatement on a bounded sample (one thread, vectorised over the batch)
    from oracle.plant_np import rk4_step
    Bc = 4096
    xc = x0[:Bc].cpu().numpy()
    uc = u[:Bc].cpu().numpy()
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_budget:
        xc = rk4_step(xc, uc[:, steps % S], 1e-3, args.substeps, bool(args.smooth))
        steps += 1
    dt = time.perf_counter() - t0
    line["cpu_baseline"] = {"value": Bc * steps / dt, "unit": "trajectory-steps/s", "cores": 1, "kind": "port",
                            "sample": f"oracle/plant_np.py, {Bc} trajectories x {steps} steps in {dt:.1f} s"}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
