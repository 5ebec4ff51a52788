"""Summarise scripts/counters.sh passes: per kernel, mean counter value per launch."""
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ctr"


def family(k):
    """the rollout kernels by role: H <= 52 fused / small-batch kernels, config 5's cell kernels"""
    if "wide_cell_fwd_kernel" in k:
        return "wide_cell_fwd"
    if "wide_bwd_fused_kernel" in k:
        return "wide_bwd_fused_l0" if ("Lb1E" in k or ", true" in k) else "wide_bwd_fused"
    for name in ("fcr_fwd_kernel", "fcr_bwd_kernel", "fcr_sfwd_kernel", "fcr_sbwd_kernel"):
        if name in k:
            return name[4:-7]
    return None


acc = {}
for f in sorted(glob.glob(f"{root}/p*/c_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = family(r["Kernel_Name"])
        if k is None:
            continue
        acc.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {sum(v) / len(v):.4g}  (n={len(v)})")
