"""Benchmark of the LSTM-surrogate training step, one JSON line per batch size.

Step = Model_NN train_model body (Model_NN/Functions.py:541-566): LSTMModel(5, 50, 4, 3) forward on a
(B, 10, 5) window batch, MSE loss, backward into every weight, AdamW (lr 1e-3, wd 0). B = 256 is the
reference's BATCH_SIZE (Model_NN/Main.py:73); larger B shows the path's throughput. Unit: windows/s.
CPU baseline: the same step on stock torch fp32 on the host (the reference's own arithmetic).
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import surrogate_torch as S  # noqa: E402


def step_fn(m, opt, X, Y, dev):
    def step():
        opt.zero_grad()
        loss = torch.nn.functional.mse_loss(m(X, dev), Y)
        loss.backward()
        opt.step()
        return loss
    return step


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, nargs="+", default=[256, 4096, 65536])
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--cpu-budget", type=float, default=5.0)
    ap.add_argument("--hidden", type=int, default=50, help="LSTM hidden size (> 52: the wide kernels, seeded weights)")
    args = ap.parse_args()
    from test_surrogate import params_for, model_for, batch
    p = params_for(args.hidden, seed=args.hidden)
    for B in args.B:
        x, t = batch(B, seed=B)
        m = model_for(p)
        opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=0.0)
        X = torch.tensor(x, dtype=torch.float32, device="cuda:0")
        Y = torch.tensor(t, dtype=torch.float32, device="cuda:0")
        step = step_fn(m, opt, X, Y, "cuda:0")
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            step()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.steps
        line = {"metric": "surrogate training windows/s", "value": B / (ms * 1e-3), "unit": "windows/s",
                "ms_per_step": ms, "dtype": "f32",
                "config": {"workload": f"LSTMModel(5,{args.hidden},4,3) MSE + AdamW step", "B": B}}
        # CPU: the reference's arithmetic (stock torch fp32 on the host), bounded
        tm = S.build(p, torch.float32)
        topt = torch.optim.AdamW(tm.parameters(), lr=1e-3, weight_decay=0.0)
        Bc = min(B, 4096)
        Xc, Yc = torch.tensor(x[:Bc], dtype=torch.float32), torch.tensor(t[:Bc], dtype=torch.float32)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_budget:
            topt.zero_grad()
            torch.nn.functional.mse_loss(tm(Xc), Yc).backward()
            topt.step()
            n += 1
        dt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": Bc * n / dt, "unit": "windows/s", "cores": torch.get_num_threads(),
                                "kind": "port", "sample": f"stock torch fp32 CPU step, B={Bc}, {n} steps in {dt:.1f} s"}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
