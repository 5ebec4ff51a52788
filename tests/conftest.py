"""Shared test setup: repo root on sys.path, the `gpu` marker, golden-fixture loaders."""
import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


def case_names():
    return sorted(os.path.basename(p)[5:-4] for p in glob.glob(os.path.join(GOLDEN, "case_*.npz")))


def load_case(name):
    c = dict(np.load(os.path.join(GOLDEN, f"case_{name}.npz")))
    wname = str(c["weights"])
    if wname.startswith("synth_"):   # large synthetic weights are stored by seed (make_golden.py)
        from tests.golden.make_golden import synth_params
        _, H, seed = wname.split("_")
        p = synth_params(int(H), int(seed))
        w = {"W_inp": p["W_inp"], "b_inp": p["b_inp"], "W_out": p["W_out"], "fcW": p["fcW"], "fcb": p["fcb"]}
        for k in range(3):
            w[f"Wih{k}"] = p["Wih"][k]
            w[f"Whh{k}"] = p["Whh"][k]
    else:
        w = dict(np.load(os.path.join(GOLDEN, f"weights_{wname}.npz")))
    params = {
        "Wih": [w[f"Wih{k}"].astype(np.float64) for k in range(3)],
        "Whh": [w[f"Whh{k}"].astype(np.float64) for k in range(3)],
        "fcW": w["fcW"].astype(np.float64), "fcb": w["fcb"].astype(np.float64),
        "W_inp": w["W_inp"].astype(np.float64), "b_inp": w["b_inp"].astype(np.float64),
        "W_out": w["W_out"].astype(np.float64),
    }
    c["noise"] = c["noise"] if c["noise"].size else None
    for k in ("B", "N", "H", "seed", "con_active", "u_saturated"):
        c[k] = int(c[k])
    c["alpha"] = float(c["alpha"])
    return c, params


def relerr(a, b):
    """max|a-b| / max|b| per tensor (the parity metric of SURVEY.md §8(d))."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.abs(b).max() if b.size else 0.0
    return float(np.abs(a - b).max() / den) if den > 0 else float(np.abs(a - b).max() if a.size else 0.0)


@pytest.fixture(params=case_names())
def golden(request):
    return (request.param,) + load_case(request.param)
