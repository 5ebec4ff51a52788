"""Throughput of the device window gather (fcr_window_gather) vs the reference-style per-item producer.

Tables: 4096 trajectories x 150 rows (T_TRAJ of the reference traces), lookback 10, features 3/1/5.
GPU: one gather of B = 65 536 shuffled samples per launch, HIP-event timed. CPU baseline: the
restated per-item producer (oracle/windows_ref.py, what DataLoader does per sample) on a bounded
sample, one thread.
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import forging_control_amd as fca  # noqa: E402
from oracle.windows_ref import concat_item  # noqa: E402


def main():
    n_traj, T, B = 4096, 150, 65536
    rng = np.random.default_rng(0)
    X = rng.standard_normal((n_traj * T, 3)).astype(np.float32)
    Y = rng.standard_normal((n_traj * T, 1)).astype(np.float32)
    Z = rng.standard_normal((n_traj * T, 5)).astype(np.float32)
    w = fca.SequenceWindows(X, Y, Z, T, 10)
    idx = torch.randperm(len(w))[:B].cuda()
    for _ in range(3):
        w.gather(idx, check=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 50
    e0.record()
    for _ in range(it):
        w.gather(idx, check=False)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    bytes_out = B * (3 + 1 + 50) * 4
    line = {"metric": "window-gather samples/s", "value": B / (ms * 1e-3), "unit": "samples/s", "ms_per_launch": ms,
            "config": {"workload": "SequenceDataset windows", "B": B, "lookback": 10, "traj_len": T},
            "hbm_write_gbs": bytes_out / (ms * 1e-3) / 1e9}
    n, t0 = 0, time.perf_counter()
    gi = idx[:20000].cpu().numpy()
    while time.perf_counter() - t0 < 5.0 and n < gi.size:
        concat_item(X, Y, Z, int(gi[n]), T, 10)
        n += 1
    dt = time.perf_counter() - t0
    line["cpu_baseline"] = {"value": n / dt, "unit": "samples/s", "cores": 1, "kind": "port",
                            "sample": f"oracle/windows_ref.py per-item producer, {n} samples in {dt:.1f} s"}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
