"""Stress check of the pipelined small-batch kernels (csrc/fcr_pipe.h): many fwd + bwd repetitions of one batch at
each window-set cap, every output compared bit for bit with the first repetition (a rare hand-off race would show as
a differing or non-finite output).
    python scripts/stress_pipe.py [--reps 2000]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import forging_control_amd as fca  # noqa: E402
from test_gpu_parity import _synth, _u0, run  # noqa: E402
from conftest import load_case  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=2000)
a = ap.parse_args()
params = load_case("ref_b15_n10")[1]
for B, N in ((15, 10), (256, 10), (100, 25)):
    X, S, _ = _synth(B, N, 77 + B)
    u0 = _u0(params, X)
    for sets in (0, 1, 2, 3, 4):
        prev = fca._native.set_small_pipe_sets(sets)
        try:
            ref = run(params, X, u0, S, N, 20.0, small_batch_limit=1 << 30)
            bad = 0
            for r in range(a.reps // (5 if B > 15 else 1)):
                o = run(params, X, u0, S, N, 20.0, small_batch_limit=1 << 30)
                for k, v in o.items():
                    if isinstance(v, np.ndarray) and not (np.array_equal(v, ref[k]) and np.isfinite(v).all()):
                        bad += 1
                        print(f"B {B} N {N} sets {sets} rep {r}: {k} differs", flush=True)
                        break
        finally:
            fca._native.set_small_pipe_sets(prev)
        print(f"B {B} N {N} sets {sets}: {a.reps // (5 if B > 15 else 1)} repetitions, {bad} differing", flush=True)
