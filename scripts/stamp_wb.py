"""Section shares of config 5's fused backward cell (layers >= 1) from an FCR_WB_STAMP=1 FCR_WB_N256=0 build
(diagnostic; the stamps are in WbG256's one-row producer):

    python scripts/stamp_wb.py lib_ab/wbstamp.so [--batch 65536] [--horizon 2]
Runs scripts/kbench.py's config-5 step with every window kept, then reads fcr_debug_wb_stamp: cycles per K step and
wave for each role's sections (consumers: barrier wait, A DMA issue, fragment reads + MFMA issue; producers: barrier
wait, input load issue, dgates incl. waiting for their inputs). The build's own run time is not the kernel's."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

ap = argparse.ArgumentParser()
ap.add_argument("lib")
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--horizon", type=int, default=2)
a = ap.parse_args()
buf = (ctypes.c_ulonglong * 16)()
sys.argv = [sys.argv[0], a.lib, "--batch", str(a.batch), "--horizon", str(a.horizon), "--hidden", "256",
            "--rounds", "1", "--keep-budget", "272000000000"]
import kbench  # noqa: E402  (imports torch: its HIP runtime must load before the library's)

lib = ctypes.CDLL(os.path.abspath(a.lib))
kbench.main()
assert lib.fcr_debug_wb_stamp(buf) == 0
v = list(buf)
for role, base, names in (("consumer", 0, ("barrier wait", "A DMA issue", "reads + MFMA issue")),
                          ("producer", 4, ("barrier wait", "input load issue", "dgates + tile writes"))):
    steps = max(v[base + 3], 1)
    tot = sum(v[base:base + 3])
    print(f"{role}: {steps} wave-steps, {tot / steps:.0f} cycles per step")
    for k, nm in enumerate(names):
        print(f"  {nm:22s} {v[base + k] / steps:8.0f} cycles/step  {100.0 * v[base + k] / max(tot, 1):5.1f} %")
