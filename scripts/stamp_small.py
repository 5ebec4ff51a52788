"""Per-wave section cycles of the small-batch backward from an FCR_STAMP=1 build (diagnostic).

    python scripts/stamp_small.py forging-control_amd/lib/libfcr_stamp.so [--batch 15]
Sections per cell: B (gradients + partial transposed product), A (next cell's recompute), reduction."""
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
ap.add_argument("--batch", type=int, default=15)
a = ap.parse_args()
sys.argv = [sys.argv[0], a.lib, "--batch", str(a.batch), "--rounds", "3"]
lib = ctypes.CDLL(os.path.abspath(a.lib))
lib.fcr_debug_stamp_offset.argtypes = [ctypes.POINTER(kbench._n.FcrDims)]
lib.fcr_debug_stamp_offset.restype = ctypes.c_size_t
state = kbench.main(return_state=True)
dims, ws = state["dims"], state["ws"]
off = lib.fcr_debug_stamp_offset(ctypes.byref(dims))
nq = 4
st = ws[off:off + nq * 64].view(torch.int64).reshape(nq, 8).cpu().numpy().astype(np.float64)
for w in range(nq):
    c = st[w, 3]
    print(f"wave {w}: cells {c:.0f}  B {st[w, 0] / c:7.0f}  A {st[w, 1] / c:7.0f}  reduce {st[w, 2] / c:7.0f}  "
          f"per cell total {(st[w, 0] + st[w, 1] + st[w, 2]) / c:7.0f}  lifetime {st[w, 4]:.3e} ({st[w, 4] / c:.0f}/cell)")
    print(f"        per window: 3 refills {st[w, 5] / 10:7.0f}  head {st[w, 7] / 10:7.0f}  3 phase prologues (A(9)) {st[w, 6] / 10:7.0f}")

nw_pad = (a.batch + 15) // 16
nw_pad = (nw_pad + 7) // 8 * 8
fo = off + nw_pad * 64
fw = ws[fo:fo + nq * 64].view(torch.int64).reshape(nq, 8).cpu().numpy().astype(np.float64)
for w in range(nq):
    c = fw[w, 3]
    print(f"forward wave {w}: cells {c:.0f}  cell {fw[w, 0] / c:7.0f}  exchange {fw[w, 1] / c:7.0f}  "
          f"refills/window {fw[w, 2] / 10:7.0f}  lifetime {fw[w, 4]:.3e} ({fw[w, 4] / c:.0f}/cell)")
    print(f"        per window: head+readout {fw[w, 5] / 10:7.0f}  refills incl. first record load {fw[w, 6] / 10:7.0f}")
