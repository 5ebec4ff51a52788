"""Where do two libfcr.so builds disagree? One batch through each, outputs snapshotted after the forward AND after the
backward (a later write into an output shows up as a change between the two), then the differing elements located.

    python scripts/ab_diff.py lib_ab/a.so lib/b.so [--batch 4096] [--precision 1]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import forging_control_amd as fca  # noqa: E402
from bench import load_weights, synth_batch  # noqa: E402
from kbench import bind  # noqa: E402

_n = fca._native


def run(lib, a, dev):
    B, N, H = a.batch, a.horizon, 50
    sim, ctrl = load_weights(dev, H)
    X, S = synth_batch(B, dev, 7)
    with torch.no_grad():
        u0 = ctrl(X).contiguous()
    dims = fca.rollout.make_dims(B, N, H, 3, 50, 20.0, precision=a.precision)
    opts = _n.make_options(None, None)
    o = ctypes.byref(opts)
    w = _n.FcrWeights()
    params = [ctrl.fc_inp.weight, ctrl.fc_inp.bias, ctrl.fc_out.weight]
    w.ctrl_w_inp, w.ctrl_b_inp, w.ctrl_w_out = (p.data_ptr() for p in params)
    for k in range(3):
        w.w_ih[k] = getattr(sim.lstm, f"weight_ih_l{k}").data_ptr()
        w.w_hh[k] = getattr(sim.lstm, f"weight_hh_l{k}").data_ptr()
    w.fc_w, w.fc_b = sim.fc.weight.data_ptr(), sim.fc.bias.data_ptr()
    nb = ctypes.c_size_t()
    lib.fcr_workspace_size(ctypes.byref(dims), o, 1, ctypes.byref(nb))
    ws = torch.full((nb.value,), 0x7f, dtype=torch.uint8, device=dev)   # recognisable fill
    f32 = dict(dtype=torch.float32, device=dev)
    outs = {k: torch.full(s if isinstance(s, tuple) else (s,), float("nan"), **f32) for k, s in
            dict(loss=(), cost=B, command=B, error=B, pred=B * N, xhat=(B, N, 4), gu0=(B, 1), gwi=(50, 3),
                 gbi=(50,), gwo=(1, 50)).items()}
    dl = torch.ones(1, **f32)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = lib.fcr_forward(ctypes.byref(dims), o, ctypes.byref(w), p(X), p(u0), p(S), None, p(outs["loss"]),
                         p(outs["cost"]), p(outs["command"]), p(outs["error"]), p(outs["pred"]), p(outs["xhat"]), 1,
                         p(ws), nb, st)
    torch.cuda.synchronize()
    fwd = {k: outs[k].cpu().numpy().copy() for k in ("loss", "cost", "pred", "xhat")}
    rc |= lib.fcr_backward(ctypes.byref(dims), o, p(X), p(S), p(outs["pred"]), p(dl), p(outs["gu0"]), p(outs["gwi"]),
                           p(outs["gbi"]), p(outs["gwo"]), p(ws), nb, st)
    torch.cuda.synchronize()
    if rc:
        raise RuntimeError(lib.fcr_last_error())
    bwd = {k: outs[k].cpu().numpy().copy() for k in outs}
    return fwd, bwd


def where(a, b):
    d = np.abs(a - b)
    bad = np.argwhere(d > 1e-6 * max(np.abs(a).max(), 1e-30))
    if bad.size == 0:
        return "identical" if np.array_equal(a, b, equal_nan=True) else "within 1e-6"
    out = {"n": int(len(bad)), "maxrel": float(d.max() / max(np.abs(a).max(), 1e-30))}
    for ax in range(bad.shape[1]):
        vals, cnt = np.unique(bad[:, ax], return_counts=True)
        out[f"axis{ax}"] = {int(v): int(c) for v, c in zip(vals[:12], cnt[:12])} if len(vals) <= 12 else \
            f"{len(vals)} distinct, min {vals.min()}, max {vals.max()}"
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=2)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--precision", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    (fa, ba), (fb, bb) = (run(bind(p), a, dev) for p in a.libs)
    rep = {"fwd": {k: where(fa[k], fb[k]) for k in fa}, "bwd": {k: where(ba[k], bb[k]) for k in ba},
           "a_changed_by_bwd": {k: where(fa[k], ba[k]) for k in fa},
           "b_changed_by_bwd": {k: where(fb[k], bb[k]) for k in fb}}
    print(json.dumps(rep, indent=1), flush=True)


if __name__ == "__main__":
    main()
