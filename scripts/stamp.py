"""Read the backward's per-wave section cycle sums from an FCR_STAMP=1 build (diagnostic).

    python scripts/stamp.py forging-control_amd/lib/libfcr_stamp.so [--batch 65536]
Sections per cell: prologue (top: scale, operands, first forward pair), region loop, epilogue."""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import kbench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("lib")
ap.add_argument("--batch", type=int, default=65536)
a = ap.parse_args()
sys.argv = [sys.argv[0], a.lib, "--batch", str(a.batch), "--rounds", "2"]
lib = ctypes.CDLL(os.path.abspath(a.lib))
lib.fcr_debug_stamp_offset.argtypes = [ctypes.POINTER(kbench._n.FcrDims)]
lib.fcr_debug_stamp_offset.restype = ctypes.c_size_t
state = kbench.main(return_state=True)
dims, ws = state["dims"], state["ws"]
off = lib.fcr_debug_stamp_offset(ctypes.byref(dims))
nw = (a.batch + 15) // 16
st = ws[off:off + nw * 64].view(torch.int64).reshape(nw, 8).cpu().numpy().astype(np.float64)
cells = st[:, 3]
print(f"waves {nw}, cells/wave {cells.mean():.0f}")
names = ["prologue", "regions", "epilogue"]
for k, nm in enumerate(names):
    print(f"  {nm:9s} {np.mean(st[:, k] / cells):9.0f} cycles/cell")
for k, nm in ((5, "window head (row grads, controller bwd)"), (6, "layer-2 image fill + barriers"), (7, "layer-1 image fill + barriers")):
    print(f"  {nm:40s} {np.mean(st[:, k]) / 10:9.0f} cycles/window")
print(f"  cell total {np.mean((st[:, 0] + st[:, 1] + st[:, 2]) / cells):9.0f} cycles/cell;"
      f" kernel wave lifetime {np.mean(st[:, 4]):.3e} cycles, {np.mean(st[:, 4] / cells):.0f} per cell")

nw_pad = (nw + 7) // 8 * 8
fw = ws[off + nw_pad * 64: off + nw_pad * 64 + nw * 64].view(torch.int64).reshape(nw, 8).cpu().numpy().astype(np.float64)
N = state["dims"].N
tot = fw[:, 4].mean()
print(f"forward: wave lifetime {tot:.3e} cycles; per window: head {fw[:, 0].mean() / N:.0f}, layer 0 "
      f"{fw[:, 1].mean() / N:.0f}, fills+barriers {fw[:, 2].mean() / N:.0f}, layers 1-2 + readout "
      f"{(tot - fw[:, 0].mean() - fw[:, 1].mean() - fw[:, 2].mean()) / N:.0f}")
print(f"forward refills per window: store drain {fw[:, 5].mean() / N:.0f}, barrier-1 skew {fw[:, 6].mean() / N:.0f}, "
      f"DMA {fw[:, 7].mean() / N:.0f}, barrier 2 {(fw[:, 2] - fw[:, 5] - fw[:, 6] - fw[:, 7]).mean() / N:.0f} cycles")
sk = fw[:, 6] / N
print("forward barrier-1 skew per window by wave slot in the workgroup:",
      " ".join(f"{sk[i::8].mean():.0f}" for i in range(8)))
l12 = (fw[:, 4] - fw[:, 0] - fw[:, 1] - fw[:, 2]) / N
print("forward layers 1-2 cycles per window by wave slot:", " ".join(f"{l12[i::8].mean():.0f}" for i in range(8)))
print("forward layer 0 cycles per window by wave slot:", " ".join(f"{(fw[:, 1] / N)[i::8].mean():.0f}" for i in range(8)))
