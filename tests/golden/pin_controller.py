"""Attempt to pin the controller forward (FNNModel, Functions.py:261-289, as NN_make_step applies it at
:1560-1613) on data the reference ships: its closed-loop trace results/Unsupervised_dataframe.txt (600 rows of
time, ref, y, y_dot, p1, p2, z, u written with %.6f by UL/Main.py:922-934, no noise: UL/Main.py:98,112) and its
trained controllers results/NN_controller_N_10_{0..9}[_noise].pt (loaded as data, weights_only=True).

NN_make_step computes u_t = s_u * FNN([y_dot_t / s_y, z_t / s_z, ref_t / s_y]) with MaxAbs scalers fit on the
training data (UL/Main.py:235-261), which the reference does not ship; the three scales are fitted here by
least squares for every shipped controller and every row alignment. A pin would leave residuals at the
%.6f rounding (5e-7). Run: python tests/golden/pin_controller.py (needs /root/reference; not a test).
Result (this container): no shipped controller reproduces the trace — see DESIGN.md §3."""
import json
import os
import sys

import numpy as np
import torch
from scipy.optimize import least_squares

R = "/root/reference/Unsupervised Learning/results/"


def fnn(sd, x):
    z = x @ sd["fc_inp.weight"].T + sd["fc_inp.bias"]
    return np.clip(np.maximum(z, 0.0) @ sd["fc_out.weight"][0], -1.0, 1.0)


def main():
    import pandas as pd
    df = pd.read_csv(R + "Unsupervised_dataframe.txt", sep="\t")
    y, zz, ref, u = (df[k].to_numpy() for k in ("y_dot", "z", "ref", "u"))
    idx = np.arange(2, len(u) - 2)
    out = []
    for name in [f"NN_controller_N_10_{i}{s}.pt" for i in range(10) for s in ("", "_noise")]:
        sd = {k: v.double().numpy() for k, v in torch.load(R + name, weights_only=True, map_location="cpu").items()}
        for lag in (-1, 0, 1):
            def res(p):
                sy, sz, su = p
                X = np.stack([y[idx + lag] / sy, zz[idx + lag] / sz, ref[idx] / sy], 1)
                return su * fnn(sd, X) - u[idx]
            r = least_squares(res, [0.6, 0.25, 0.25], bounds=([0.05, 0.01, 0.01], [10, 10, 10]))
            out.append({"controller": name, "state_lag": lag, "scales": [float(v) for v in r.x],
                        "max_abs_residual": float(np.abs(r.fun).max()),
                        "median_abs_residual": float(np.median(np.abs(r.fun))),
                        "rms_residual": float(np.sqrt(np.mean(r.fun ** 2)))})
    out.sort(key=lambda d: d["rms_residual"])
    json.dump({"rounding": 5e-7, "best": out[:5]}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
