"""NumPy restatement of the batched closed loop (TEST INFRASTRUCTURE ONLY).

Per step, as NeuralNetwork.loop (Functions.py:1116-1200) without feasibility recovery and noise:
NN_make_step (Functions.py:1594-1604) — MaxAbs-scaled [y_dot, z, ref] in fp64 (the reference column by
scalers['y_dot']), the FNN in float32 as torch runs it (Linear+ReLU, Linear without bias, Hardtanh),
unscaled by scalers['output'] in float32 — then the plant step of oracle/plant_np.py (RK4 of
Functions.py:1743-1781). PARITY STATUS: composed of restatements pinned elsewhere (plant_np: the
reference's traces; the FNN: the rollout oracle's fixtures); the loop order follows the reference.
"""
from __future__ import annotations

import numpy as np

from .plant_np import rk4_step


def controller_u(x, ref, W_inp, b_inp, W_out, in_scale, ref_scale, out_scale):
    f32 = np.float32
    s = np.stack([x[:, 1] / in_scale[0], x[:, 4] / in_scale[1], ref / ref_scale], axis=1).astype(f32)
    h = np.maximum(s @ W_inp.astype(f32).T + b_inp.astype(f32), f32(0))
    v = np.clip(h @ W_out.astype(f32).T, f32(-1), f32(1))[:, 0]
    return (v * f32(out_scale)).astype(np.float64)


def closed_loop(x0, ref, W_inp, b_inp, W_out, in_scale, ref_scale, out_scale, ts=1e-3, substeps=4, smooth=True):
    x = np.asarray(x0, np.float64)
    B, T = ref.shape
    xs = np.empty((B, T + 1, 5))
    us = np.empty((B, T))
    xs[:, 0] = x
    for t in range(T):
        u = controller_u(x, ref[:, t], W_inp, b_inp, W_out, in_scale, ref_scale, out_scale)
        x = rk4_step(x, u, ts, substeps, smooth)
        us[:, t] = u
        xs[:, t + 1] = x
    return xs, us
