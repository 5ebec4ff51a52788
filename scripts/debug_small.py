"""Diagnostic: small-batch vs fused backward on the same forward (FCR_STAMP build): first differing dseq cell.
    python scripts/debug_small.py forging-control_amd/lib/libfcr_stamp.so --hidden 32 --batch 16 --horizon 6"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import forging_control_amd as fca  # noqa: E402
from bench import load_weights, synth_batch  # noqa: E402

_n = fca._native
ap = argparse.ArgumentParser()
ap.add_argument("lib")
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--horizon", type=int, default=6)
ap.add_argument("--hidden", type=int, default=32)
a = ap.parse_args()
lib = ctypes.CDLL(os.path.abspath(a.lib))
vp, i32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
D = ctypes.POINTER(_n.FcrDims)
lib.fcr_workspace_size.argtypes = [D, i32, ctypes.POINTER(sz)]
lib.fcr_forward.argtypes = [D, ctypes.POINTER(_n.FcrWeights)] + [vp] * 10 + [i32, vp, sz, vp]
lib.fcr_backward.argtypes = [D] + [vp] * 8 + [vp, sz, vp]
lib.fcr_set_small_batch_limit.argtypes = [i32]
for f in ("fcr_debug_dseq_offset", "fcr_debug_dxrow_offset"):
    getattr(lib, f).argtypes = [D]
    getattr(lib, f).restype = sz
dev = torch.device("cuda", 0)
B, N, H = a.batch, a.horizon, a.hidden
sim, ctrl = load_weights(dev, H)
X, S = synth_batch(B, dev, 7)
with torch.no_grad():
    u0 = ctrl(X).contiguous()
dims = fca.rollout.make_dims(B, N, H, 3, 50, 20.0)
w = _n.FcrWeights()
w.ctrl_w_inp, w.ctrl_b_inp, w.ctrl_w_out = (p.data_ptr() for p in (ctrl.fc_inp.weight, ctrl.fc_inp.bias, ctrl.fc_out.weight))
for k in range(3):
    w.w_ih[k] = getattr(sim.lstm, f"weight_ih_l{k}").data_ptr()
    w.w_hh[k] = getattr(sim.lstm, f"weight_hh_l{k}").data_ptr()
w.fc_w, w.fc_b = sim.fc.weight.data_ptr(), sim.fc.bias.data_ptr()
nb = ctypes.c_size_t()
lib.fcr_workspace_size(ctypes.byref(dims), 1, ctypes.byref(nb))
ws = torch.zeros(nb.value, dtype=torch.uint8, device=dev)
f32 = dict(dtype=torch.float32, device=dev)
o = {k: torch.zeros(s, **f32) for k, s in dict(loss=(), cost=B, command=B, error=B, pred=B * N, xhat=(B, N, 4),
                                               gu0=(B, 1), gwi=(50, 3), gbi=(50,), gwo=(1, 50)).items()}
dl = torch.ones(1, **f32)
p = lambda t: ctypes.c_void_p(t.data_ptr())
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
lib.fcr_set_small_batch_limit(1 << 30)
assert lib.fcr_forward(ctypes.byref(dims), ctypes.byref(w), p(X), p(u0), p(S), None, p(o["loss"]), p(o["cost"]),
                       p(o["command"]), p(o["error"]), p(o["pred"]), p(o["xhat"]), 1, p(ws), nb, st) == 0
HS = 4 if H <= 16 else (8 if H <= 32 else 13)
qc = HS * 16 * 16   # bytes per cell record
off = lib.fcr_debug_dseq_offset(ctypes.byref(dims))
offr = lib.fcr_debug_dxrow_offset(ctypes.byref(dims))
res = {}
for lim in (0, 1 << 30):
    lib.fcr_set_small_batch_limit(lim)
    ws[off:off + N * 2 * 10 * qc].zero_()
    assert lib.fcr_backward(ctypes.byref(dims), p(X), p(S), p(o["pred"]), p(dl), p(o["gu0"]), p(o["gwi"]), p(o["gbi"]),
                            p(o["gwo"]), p(ws), nb, st) == 0
    torch.cuda.synchronize()
    d = ws[off:off + N * 2 * 10 * qc].view(torch.float32).cpu().numpy().reshape(N, 2, 10, -1).copy()
    r = ws[offr:offr + N * 10 * 64 * 8].view(torch.float32).cpu().numpy().reshape(N, 10, 64, 2).copy()
    res[lim] = (d, r, o["gu0"].cpu().numpy().copy(), o["gwi"].cpu().numpy().copy())
(d0, r0, g0, w0), (d1, r1, g1, w1) = res[0], res[1 << 30]
print("g_u0 rel", np.abs(g0 - g1).max() / np.abs(g0).max(), "g_W_inp rel", np.abs(w0 - w1).max() / np.abs(w0).max())
for j in range(N - 1, -1, -1):
    for li, l in enumerate((2, 1)):
        for t in range(9, -1, -1):
            a_, b_ = d0[j, li, t], d1[j, li, t]
            e = np.abs(a_ - b_).max() / max(np.abs(a_).max(), 1e-30)
            if e > 1e-5:
                print(f"dseq window {j} from layer {l} t {t}: rel {e:.3e} (max {np.abs(a_).max():.3e})")
                qa, qb = a_.reshape(-1, 64, 4), b_.reshape(-1, 64, 4)
                print("   per quad:", [float(np.abs(qa[k] - qb[k]).max()) for k in range(qa.shape[0])],
                      "per lane group:", [float(np.abs(qa[:, 16 * g:16 * g + 16] - qb[:, 16 * g:16 * g + 16]).max()) for g in range(4)])
    for t in range(9, -1, -1):
        a_, b_ = r0[j, t], r1[j, t]
        e = np.abs(a_ - b_).max() / max(np.abs(a_).max(), 1e-30)
        if e > 1e-5:
            print(f"dxrow window {j} t {t}: rel {e:.3e}")
