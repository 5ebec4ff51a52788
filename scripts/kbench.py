"""A/B timing of libfcr.so build variants in ONE process (interleaved rounds, same device, same data).

    python scripts/kbench.py lib/a.so lib/b.so ... [--batch 65536] [--rounds 5]

For each variant: fcr_forward(with_backward=1) and fcr_backward timed with HIP events on the launch
stream; outputs are checked against the first variant (loss, g_u0, controller grads within 1e-5 rel).
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
import forging_control_amd as fca  # noqa: E402
from bench import load_weights, synth_batch  # noqa: E402

_n = fca._native


class _V4:
    """An ABI v4 library (round 3: no fcr_options argument) behind the v5 call signatures used below."""

    def __init__(self, lib):
        self.lib = lib

    def fcr_workspace_size(self, d, o, wb, nb):
        return self.lib.fcr_workspace_size(d, wb, nb)

    def fcr_forward(self, d, o, *rest):
        return self.lib.fcr_forward(d, *rest)

    def fcr_backward(self, d, o, *rest):
        return self.lib.fcr_backward(d, *rest)

    def fcr_last_error(self):
        return self.lib.fcr_last_error()


def bind(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    vp, i32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    lib.fcr_last_error.restype = ctypes.c_char_p
    if lib.fcr_abi_version() < 5:   # round-3 builds: the same calls without the options pointer
        lib.fcr_workspace_size.argtypes = [ctypes.POINTER(_n.FcrDims), i32, ctypes.POINTER(sz)]
        lib.fcr_forward.argtypes = [ctypes.POINTER(_n.FcrDims), ctypes.POINTER(_n.FcrWeights)] + [vp] * 10 + [i32, vp, sz, vp]
        lib.fcr_backward.argtypes = [ctypes.POINTER(_n.FcrDims)] + [vp] * 8 + [vp, sz, vp]
        return _V4(lib)
    po = ctypes.POINTER(_n.FcrOptions)   # ABI v5 (include/fcr.h)
    lib.fcr_workspace_size.argtypes = [ctypes.POINTER(_n.FcrDims), po, i32, ctypes.POINTER(sz)]
    lib.fcr_forward.argtypes = [ctypes.POINTER(_n.FcrDims), po, ctypes.POINTER(_n.FcrWeights)] + [vp] * 10 + [i32, vp, sz, vp]
    lib.fcr_backward.argtypes = [ctypes.POINTER(_n.FcrDims), po] + [vp] * 8 + [vp, sz, vp]
    return lib


def main(return_state=False):
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--hidden", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--sustain", type=int, default=0, help="then time this many back-to-back launches per lib")
    ap.add_argument("--precision", type=int, default=0, help="0 = fp32-accurate, 1 = f16 (config 3)")
    ap.add_argument("--keep-budget", type=int, default=None,
                    help="fcr_options.wide_keep_budget bytes (H > 52: kept windows skip the backward recompute)")
    ap.add_argument("--small-limit", type=int, default=None, help="fcr_options.small_batch_limit")
    a = ap.parse_args()
    opts = _n.make_options(a.small_limit, a.keep_budget)
    o = ctypes.byref(opts)
    dev = torch.device("cuda", 0)
    B, N, H = a.batch, a.horizon, a.hidden
    sim, ctrl = load_weights(dev, H)
    X, S = synth_batch(B, dev, 7)
    with torch.no_grad():
        u0 = ctrl(X).contiguous()
    dims = fca.rollout.make_dims(B, N, H, 3, 50, 20.0, precision=a.precision)
    w = _n.FcrWeights()
    params = [ctrl.fc_inp.weight, ctrl.fc_inp.bias, ctrl.fc_out.weight]
    w.ctrl_w_inp, w.ctrl_b_inp, w.ctrl_w_out = (p.data_ptr() for p in params)
    for k in range(3):
        w.w_ih[k] = getattr(sim.lstm, f"weight_ih_l{k}").data_ptr()
        w.w_hh[k] = getattr(sim.lstm, f"weight_hh_l{k}").data_ptr()
    w.fc_w, w.fc_b = sim.fc.weight.data_ptr(), sim.fc.bias.data_ptr()
    libs = [bind(p) for p in a.libs]
    for lib in libs:   # ABI v4 builds take the keep budget / small-batch limit process-wide
        if isinstance(lib, _V4) and a.keep_budget is not None:
            lib.lib.fcr_set_wide_keep_budget.argtypes = [ctypes.c_int64]
            lib.lib.fcr_set_wide_keep_budget(a.keep_budget)
        if isinstance(lib, _V4) and a.small_limit is not None:
            lib.lib.fcr_set_small_batch_limit(a.small_limit)
    need = []
    for lib in libs:
        nb = ctypes.c_size_t()
        lib.fcr_workspace_size(ctypes.byref(dims), o, 1, ctypes.byref(nb))
        need.append(nb.value)
    nbytes = ctypes.c_size_t(max(need))
    print(f"# workspace {nbytes.value / 2**30:.1f} GiB", flush=True)
    ws = torch.empty(nbytes.value, dtype=torch.uint8, device=dev)
    f32 = dict(dtype=torch.float32, device=dev)
    outs = {k: torch.empty(s, **f32) for k, s in
            dict(loss=(), cost=B, command=B, error=B, pred=B * N, xhat=(B, N, 4), gu0=(B, 1), gwi=(50, 3),
                 gbi=(50,), gwo=(1, 50)).items()}
    dl = torch.ones(1, **f32)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    times = {i: {"fwd": [], "bwd": []} for i in range(len(libs))}
    ref = None
    results = {}
    for rnd in range(a.rounds + 1):
        for i, lib in enumerate(libs):
            ev[0].record()
            rc = lib.fcr_forward(ctypes.byref(dims), o, ctypes.byref(w), p(X), p(u0), p(S), None, p(outs["loss"]),
                                 p(outs["cost"]), p(outs["command"]), p(outs["error"]), p(outs["pred"]),
                                 p(outs["xhat"]), 1, p(ws), nbytes, st)
            ev[1].record()
            rc |= lib.fcr_backward(ctypes.byref(dims), o, p(X), p(S), p(outs["pred"]), p(dl), p(outs["gu0"]),
                                   p(outs["gwi"]), p(outs["gbi"]), p(outs["gwo"]), p(ws), nbytes, st)
            ev[2].record()
            torch.cuda.synchronize()
            if rc:
                raise RuntimeError(lib.fcr_last_error())
            if rnd > 0:
                times[i]["fwd"].append(ev[0].elapsed_time(ev[1]))
                times[i]["bwd"].append(ev[1].elapsed_time(ev[2]))
            snap = {k: outs[k].detach().cpu().numpy().copy() for k in ("loss", "gu0", "gwi", "gbi", "gwo", "xhat")}
            if ref is None:
                ref = snap
            results[i] = {k: float(np.abs(snap[k] - ref[k]).max() / max(np.abs(ref[k]).max(), 1e-30)) for k in snap}
    if a.sustain:
        # back-to-back launches with no host sync (the clock the chip holds under sustained load)
        for i, lib in enumerate(libs):
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.sustain + 1)]
            evs[0].record()
            for k in range(a.sustain):
                lib.fcr_forward(ctypes.byref(dims), o, ctypes.byref(w), p(X), p(u0), p(S), None, p(outs["loss"]),
                                p(outs["cost"]), p(outs["command"]), p(outs["error"]), p(outs["pred"]),
                                p(outs["xhat"]), 1, p(ws), nbytes, st)
                evs[2 * k + 1].record()
                lib.fcr_backward(ctypes.byref(dims), o, p(X), p(S), p(outs["pred"]), p(dl), p(outs["gu0"]),
                                 p(outs["gwi"]), p(outs["gbi"]), p(outs["gwo"]), p(ws), nbytes, st)
                evs[2 * k + 2].record()
            torch.cuda.synchronize()
            h = a.sustain // 2
            times[i]["fwd"] = [evs[2 * k].elapsed_time(evs[2 * k + 1]) for k in range(h, a.sustain)]
            times[i]["bwd"] = [evs[2 * k + 1].elapsed_time(evs[2 * k + 2]) for k in range(h, a.sustain)]
    if return_state:
        return {"dims": dims, "ws": ws}
    for i, path in enumerate(a.libs):
        f, b = np.median(times[i]["fwd"]), np.median(times[i]["bwd"])
        print(json.dumps({"lib": os.path.basename(path), "fwd_ms": round(f, 3), "bwd_ms": round(b, 3),
                          "fwd_min": round(min(times[i]["fwd"]), 3), "bwd_min": round(min(times[i]["bwd"]), 3),
                          "step_ms": round(f + b, 3), "maxrel_vs_first": max(results[i].values()),
                          "maxrel_by_output": {k: float(f"{v:.3g}") for k, v in results[i].items()}}), flush=True)


if __name__ == "__main__":
    main()
