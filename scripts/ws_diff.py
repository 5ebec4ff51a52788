"""Diagnostic: run fcr_forward + fcr_backward of two builds with the SAME workspace layout on the same inputs (one
process, one device) and report, per 1 MiB block of the workspace, the largest relative difference after the
backward — where two builds' intermediate buffers part ways.   python scripts/ws_diff.py a.so b.so"""
import ctypes
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
dev = torch.device("cuda", 0)
B, N, H = int(os.environ.get("WSB", 8)), 25, 256
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
libs = [bind(p) for p in sys.argv[1:3]]
sizes = []
for lib in libs:
    nb = ctypes.c_size_t()
    assert lib.fcr_workspace_size(ctypes.byref(dims), None, 1, ctypes.byref(nb)) == 0
    sizes.append(nb.value)
print("workspace sizes", sizes)
f32 = dict(dtype=torch.float32, device=dev)
p = lambda t: ctypes.c_void_p(t.data_ptr())
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
snaps, outs = [], []
for lib in libs:
    ws = torch.zeros(max(sizes), dtype=torch.uint8, device=dev)
    o = {k: torch.zeros(s, **f32) for k, s in dict(loss=(), cost=B, command=B, error=B, pred=B * N, xhat=(B, N, 4),
                                                   gu0=(B, 1), gwi=(50, 3), gbi=(50,), gwo=(1, 50)).items()}
    dl = torch.ones(1, **f32)
    rc = lib.fcr_forward(ctypes.byref(dims), None, ctypes.byref(w), p(X), p(u0), p(S), None, p(o["loss"]), p(o["cost"]),
                         p(o["command"]), p(o["error"]), p(o["pred"]), p(o["xhat"]), 1, p(ws), ws.numel(), st)
    rc |= lib.fcr_backward(ctypes.byref(dims), None, p(X), p(S), p(o["pred"]), p(dl), p(o["gu0"]), p(o["gwi"]), p(o["gbi"]),
                           p(o["gwo"]), p(ws), ws.numel(), st)
    torch.cuda.synchronize()
    assert rc == 0, lib.fcr_last_error()
    snaps.append(ws.cpu().numpy())
    outs.append({k: v.cpu().numpy() for k, v in o.items()})
for k in outs[0]:
    a, b = outs[0][k], outs[1][k]
    print(k, float(np.abs(a - b).max() / max(np.abs(a).max(), 1e-30)))
A = snaps[0][: (min(sizes) // 4) * 4].view(np.float32)
Bv = snaps[1][: (min(sizes) // 4) * 4].view(np.float32)
blk = 1 << 18   # floats per 1 MiB
for i in range(0, A.size, blk):
    a, b = A[i:i + blk], Bv[i:i + blk]
    m = np.isfinite(a) & np.isfinite(b)
    if not m.any():
        continue
    d = np.abs(a[m] - b[m]).max()
    s = np.abs(a[m]).max()
    if d > 1e-5 * max(s, 1e-30):
        print(f"MiB {i // blk:6d}: max|diff| {d:.3e} max|a| {s:.3e}  first differing float at byte {4 * (i + int(np.argmax(np.abs(a - b) > 1e-5 * s)))}")
off = int(os.environ.get("WSD0", 0))
if off:
    n = 10 * B * 2 * H
    a = A[off // 4: off // 4 + n].reshape(10, B, 2 * H)
    b = Bv[off // 4: off // 4 + n].reshape(10, B, 2 * H)
    for t in range(10):
        for part in (0, 1):
            x, y = a[t, :, part * H:(part + 1) * H], b[t, :, part * H:(part + 1) * H]
            print(f"D0 t={t} part={part}: max|a| {np.abs(x).max():.3e} max|b| {np.abs(y).max():.3e} rel diff {np.abs(x - y).max() / max(np.abs(x).max(), 1e-30):.3e}")
if off:
    np.save(os.path.join(ROOT, "gpurun_out", "r3i", "d0_a.npy"), a)
    np.save(os.path.join(ROOT, "gpurun_out", "r3i", "d0_b.npy"), b)
    np.save(os.path.join(ROOT, "gpurun_out", "r3i", "d1_a.npy"), A[(off + 163840) // 4:(off + 163840) // 4 + n].reshape(10, B, 2 * H))
    np.save(os.path.join(ROOT, "gpurun_out", "r3i", "d1_b.npy"), Bv[(off + 163840) // 4:(off + 163840) // 4 + n].reshape(10, B, 2 * H))
