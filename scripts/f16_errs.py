"""f16-mode (config 3) errors against the fp64 oracle fixtures, per output (the numbers tests/test_gpu_precision.py
bounds), for the library in forging-control_amd/lib."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
from conftest import case_names, load_case, relerr  # noqa: E402
import test_gpu_parity as T  # noqa: E402
from test_gpu_precision import run_p  # noqa: E402

for name in case_names():
    c, params = load_case(name)
    if c["H"] > 52:
        continue
    o = run_p(params, c, "f16")
    errs = {k: relerr(o[k], c[f"{k}_64"]) for k in T.FEATS + ("xhat",) + tuple(k for k, _ in T.GRADS)}
    print(json.dumps({"case": name, **{k: float(f"{v:.3g}") for k, v in errs.items()}}), flush=True)
