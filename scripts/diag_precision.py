"""Errors of the f16 precision mode vs the fp64 oracle on every golden case with H <= 52 (diagnostic)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch
import forging_control_amd as fca
from conftest import case_names, load_case, relerr
import test_gpu_parity as T

def run_p(params, c, precision):
    sim, ctrl = T.modules(params)
    d = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=T.DEV)
    u0_t = d(c["u0"]).reshape(-1, 1).requires_grad_(True)
    fn = fca.MPCLoss(prediction_horizon=c["N"], alpha=c["alpha"], precision=precision)
    loss, feats = fn(sim, ctrl, d(c["X"]), u0_t, d(c["states"]), T.DEV, enable_noise=c["noise"] is not None,
                     noise=None if c["noise"] is None else d(c["noise"]))
    loss.backward()
    out = {k: v.detach().cpu().numpy() for k, v in feats.items()}
    out["xhat"] = fn.last_trajectory.cpu().numpy()
    out["g_u0"] = u0_t.grad.reshape(-1).cpu().numpy()
    for k, name in T.GRADS[1:]:
        mod, attr = name.split(".")
        out[k] = getattr(getattr(ctrl, mod), attr).grad.cpu().numpy()
    return out

worst = {}
for name in case_names():
    c, params = load_case(name)
    if c["H"] > 52: continue
    o = run_p(params, c, "f16")
    errs = {k: relerr(o[k], c[f"{k}_64"]) for k in T.FEATS + ("xhat",) + tuple(g for g, _ in T.GRADS)}
    print(name, " ".join(f"{k}={v:.1e}" for k, v in errs.items()))
    for k, v in errs.items(): worst[k] = max(worst.get(k, 0), v)
print("WORST", " ".join(f"{k}={v:.1e}" for k, v in worst.items()))
