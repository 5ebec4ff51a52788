"""NumPy restatement of the batched closed loop (TEST INFRASTRUCTURE ONLY).

Per step, as NeuralNetwork.loop (Functions.py:1116-1200) without feasibility recovery and noise:
NN_make_step (Functions.py:1594-1604) — MaxAbs-scaled [y_dot, z, ref] in fp64 (the reference column by
scalers['y_dot']), the FNN in float32 (Linear+ReLU, Linear without bias, Hardtanh; the kernel's FMA order),
unscaled by scalers['output'] in float32 — then the plant step of oracle/plant_np.py (RK4 of
Functions.py:1743-1781). PARITY STATUS: composed of restatements pinned elsewhere (plant_np: the
reference's traces; the FNN: the rollout oracle's fixtures); the loop order follows the reference.
"""
from __future__ import annotations

import numpy as np

from .plant_np import rk4_step


def _fma32(a, b, c):
    """float32 fused multiply-add: the float32 x float32 product is exact in float64, the sum is rounded
    once to float64 and then to float32 (a double rounding that differs from fmaf only in vanishingly
    rare ties)."""
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


def controller_u(x, ref, W_inp, b_inp, W_out, in_scale, ref_scale, out_scale):
    """u = scalers['output'].inverse_transform(FNN(float32(X_new))) (Functions.py:1594-1604), the float32
    dot products accumulated in the kernel's order (one FMA chain per hidden unit, then over units) so the
    closed loop is compared free of summation-order noise."""
    f32 = np.float32
    s0 = (x[:, 1] / in_scale[0]).astype(f32)
    s1 = (x[:, 4] / in_scale[1]).astype(f32)
    s2 = (ref / ref_scale).astype(f32)
    W_inp, b_inp, W_out = W_inp.astype(f32), b_inp.astype(f32), W_out.astype(f32)
    v = np.zeros_like(s0)
    for j in range(W_inp.shape[0]):
        z = _fma32(np.full_like(s0, W_inp[j, 0]), s0, np.full_like(s0, b_inp[j]))
        z = _fma32(np.full_like(s0, W_inp[j, 1]), s1, z)
        z = _fma32(np.full_like(s0, W_inp[j, 2]), s2, z)
        v = _fma32(np.full_like(s0, W_out[0, j]), np.maximum(z, f32(0)), v)
    v = np.clip(v, f32(-1), f32(1))
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
