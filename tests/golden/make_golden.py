"""Generate the committed golden fixtures for the rollout parity tests.

Run in the build container (needs /root/reference for the trained weights; the GPU box only reads
the committed .npz files):

    python tests/golden/make_golden.py

Weights: the reference's own trained artifacts, loaded as DATA with ``torch.load(weights_only=True)``:
  * LSTM surrogate  ``Unsupervised Learning/Model_NN/results/model_NN.pt`` (and ``model_NN_noise.pt``)
  * controller      ``Unsupervised Learning/results/NN_controller_N_10_0.pt`` (and ``..._noise.pt``)
plus seeded synthetic weights for H in {16, 32}. Inputs are seeded synthetic tensors with the
distribution of SURVEY.md §8(d) (the reference's Data/ pickle is not shipped). Expected outputs come
from BOTH oracle restatements (fp64 NumPy with a hand-written reverse pass, and stock-torch autograd
in fp64 and fp32); the script refuses to write a fixture unless the two fp64 restatements agree to
1e-10 relative. Parity status: unpinned by reference tests (there are none) — see DESIGN.md.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import rollout_np as R  # noqa: E402
from oracle import rollout_torch as T  # noqa: E402

REF = "/root/reference/Unsupervised Learning"
OUT = os.path.dirname(os.path.abspath(__file__))
ALPHA = 20.0  # UL/Main.py:192


def load_ref_params(noise: bool):
    sfx = "_noise" if noise else ""
    lstm = torch.load(f"{REF}/Model_NN/results/model_NN{sfx}.pt", weights_only=True, map_location="cpu")
    ctrl = torch.load(f"{REF}/results/NN_controller_N_10_0{sfx}.pt", weights_only=True, map_location="cpu")
    f64 = lambda t: t.detach().double().numpy()
    return {
        "Wih": [f64(lstm[f"lstm.weight_ih_l{k}"]) for k in range(3)],
        "Whh": [f64(lstm[f"lstm.weight_hh_l{k}"]) for k in range(3)],
        "fcW": f64(lstm["fc.weight"]), "fcb": f64(lstm["fc.bias"]),
        "W_inp": f64(ctrl["fc_inp.weight"]), "b_inp": f64(ctrl["fc_inp.bias"]), "W_out": f64(ctrl["fc_out.weight"]),
    }


def synth_params(H, seed, ctrl_hidden=50):
    g = np.random.default_rng(seed)
    k = 1.0 / np.sqrt(H)   # torch's LSTM init range
    u = lambda *s: g.uniform(-k, k, s).astype(np.float32).astype(np.float64)
    xn = lambda fo, fi: (g.normal(0, np.sqrt(2.0 / (fo + fi)), (fo, fi))).astype(np.float32).astype(np.float64)
    return {
        "Wih": [u(4 * H, 5), u(4 * H, H), u(4 * H, H)],
        "Whh": [u(4 * H, H), u(4 * H, H), u(4 * H, H)],
        "fcW": u(4, H), "fcb": u(4),
        "W_inp": xn(ctrl_hidden, 3), "b_inp": g.uniform(-0.05, 0.05, ctrl_hidden).astype(np.float32).astype(np.float64),
        "W_out": xn(1, ctrl_hidden),
    }


def synth_inputs(B, N, seed, wide=False, noise=False):
    """X = [y_dot, z, ref], y_dot,z ~ U(-1,1), ref = +-U(0.11,0.99); states rows
    [y_dot,p1,p2,z,u] with y_dot,z,u ~ U(-1,1), p1,p2 ~ U(0,1.1). `wide` stretches the pressures so the
    constraint branches (Functions.py:1411) fire and the controller saturates."""
    g = np.random.default_rng(seed)
    X = np.empty((B, 3))
    X[:, 0] = g.uniform(-1, 1, B)
    X[:, 1] = g.uniform(-1, 1, B)
    X[:, 2] = g.choice([-1.0, 1.0], B) * g.uniform(0.11, 0.99, B)
    S = np.empty((B, 10, 5))
    S[:, :, [0, 3, 4]] = g.uniform(-1, 1, (B, 10, 3))
    lo, hi = (-1.5, 3.5) if wide else (0.0, 1.1)
    S[:, :, 1:3] = g.uniform(lo, hi, (B, 10, 2))
    if wide:
        S[:, :, 0] *= 3.0
        X[:, :2] *= 3.0
    nz = (g.standard_normal((B, N, 4)) * 0.01) if noise else None
    f32 = lambda a: None if a is None else a.astype(np.float32)
    return f32(X), f32(S), f32(nz)


def controller_u0(params, X):
    """u0 = controller(X) in fp32 (UL/Functions.py:643), used as the given input of the loss."""
    _, ctrl = T.build_modules(params, torch.float32)
    with torch.no_grad():
        return ctrl(torch.as_tensor(X)).numpy().astype(np.float32)


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def make_case(name, params, B, N, seed, wide=False, noise=False):
    X, S, nz = synth_inputs(B, N, seed, wide, noise)
    u0 = controller_u0(params, X).reshape(B)
    loss, feats, tape = R.rollout_forward(params, X, u0, S, N, ALPHA, None if nz is None else nz.astype(np.float64))
    grads = R.rollout_backward(params, tape)
    t64 = T.loss_and_grads(params, X, u0, S, N, ALPHA, nz, dtype=torch.float64)
    t32 = T.loss_and_grads(params, X, u0, S, N, ALPHA, nz, dtype=torch.float32)
    worst = 0.0
    for k in ("loss", "command", "error", "prediction", "xhat"):
        worst = max(worst, rel(feats[k], t64[k]))
    for k in grads:
        worst = max(worst, rel(grads[k], t64[k]))
    assert worst < 1e-10, f"{name}: fp64 restatements disagree ({worst:.3e})"
    out = {
        "B": B, "N": N, "H": params["Whh"][0].shape[1], "alpha": ALPHA, "seed": seed,
        "X": X, "u0": u0.astype(np.float32), "states": S,
        "noise": nz if nz is not None else np.zeros((0,), np.float32),
        "loss64": np.float64(loss), "loss32": t32["loss_scalar"].astype(np.float32),
    }
    for k in ("loss", "command", "error", "prediction", "xhat"):
        out[f"{k}_64"] = feats[k]
        out[f"{k}_32"] = t32[k].astype(np.float32)
    for k in grads:
        out[f"{k}_64"] = grads[k]
        out[f"{k}_32"] = t32[k].astype(np.float32)
    # branch coverage of the fixture (printed; tests assert the stress cases hit them)
    xh = feats["xhat"]
    cover = {
        "con_active": int(((xh[..., 1] < 0) | (xh[..., 1] > R.P1_MAX) | (xh[..., 2] < 0) | (xh[..., 2] > R.P2_MAX)).sum()),
        "u_saturated": int((np.abs(feats["prediction"]) >= 1.0).sum()),
        "fp32_vs_fp64": max(rel(t32[k], feats[k]) for k in ("loss", "prediction", "xhat")),
        "fp32_grad_vs_fp64": max(rel(t32[k], grads[k]) for k in grads),
    }
    out["con_active"] = cover["con_active"]
    out["u_saturated"] = cover["u_saturated"]
    print(f"{name}: B={B} N={N} H={out['H']} loss={loss:.6f} worst64={worst:.1e} {cover}")
    return out


def pack_params(params):
    d = {"W_inp": params["W_inp"], "b_inp": params["b_inp"], "W_out": params["W_out"],
         "fcW": params["fcW"], "fcb": params["fcb"]}
    for k in range(3):
        d[f"Wih{k}"] = params["Wih"][k]
        d[f"Whh{k}"] = params["Whh"][k]
    return {k: np.asarray(v, np.float32) for k, v in d.items()}


# Cases whose weights are synthetic and large are stored by seed, not by value: "synth_<H>_<seed>"
# names synth_params(H, seed) (conftest.load_case regenerates them; float32-exact by construction).
SYNTH_CASES = {
    "h64_b24_n3": (64, 11, 24, 3, 11, False),
    "h256_b8_n25": (256, 9, 8, 25, 9, False),       # SURVEY §8(c)/(d) config 5 shape at B = 8
}


def make_synth_cases(only=None):
    for name, (H, pseed, B, N, seed, wide) in SYNTH_CASES.items():
        if only and name not in only:
            continue
        c = make_case(name, synth_params(H, pseed), B, N, seed, wide=wide)
        c["weights"] = f"synth_{H}_{pseed}"
        np.savez_compressed(os.path.join(OUT, f"case_{name}.npz"), **{k: np.asarray(v) for k, v in c.items()})


def main():
    torch.set_num_threads(8)
    if len(sys.argv) > 2 and sys.argv[1] == "--only":
        make_synth_cases(set(sys.argv[2:]))
        return
    make_synth_cases()
    ref = load_ref_params(False)
    refn = load_ref_params(True)
    h16 = synth_params(16, 7)
    h32 = synth_params(32, 8)
    cases = {
        "ref_b15_n10": make_case("ref_b15_n10", ref, 15, 10, 0),             # UL plumbing batch 150//N
        "ref_b256_n10": make_case("ref_b256_n10", ref, 256, 10, 1),           # BASELINE config 1 as written
        "ref_b1_n1": make_case("ref_b1_n1", ref, 1, 1, 2),
        "ref_b3_n2": make_case("ref_b3_n2", ref, 3, 2, 3),
        "ref_b37_n25": make_case("ref_b37_n25", ref, 37, 25, 4),              # N=25 horizon, ragged batch
        "ref_wide_b64_n10": make_case("ref_wide_b64_n10", ref, 64, 10, 5, wide=True),
        "refnoise_b15_n10": make_case("refnoise_b15_n10", refn, 15, 10, 6, noise=True),
        "h16_b33_n4": make_case("h16_b33_n4", h16, 33, 4, 7, wide=True),
        "h32_b16_n6": make_case("h32_b16_n6", h32, 16, 6, 8),
    }
    params = {"ref": ref, "refnoise": refn, "h16": h16, "h32": h32}
    pmap = {"ref_b15_n10": "ref", "ref_b256_n10": "ref", "ref_b1_n1": "ref", "ref_b3_n2": "ref",
            "ref_b37_n25": "ref", "ref_wide_b64_n10": "ref", "refnoise_b15_n10": "refnoise",
            "h16_b33_n4": "h16", "h32_b16_n6": "h32"}
    for name, p in params.items():
        np.savez_compressed(os.path.join(OUT, f"weights_{name}.npz"), **pack_params(p))
    for name, c in cases.items():
        c["weights"] = pmap[name]
        np.savez_compressed(os.path.join(OUT, f"case_{name}.npz"), **{k: np.asarray(v) for k, v in c.items()})
    print("wrote", len(cases), "cases to", OUT)


if __name__ == "__main__":
    main()
