"""Summarise scripts/counters.sh passes: per kernel, mean counter value per launch."""
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ctr"
wide = len(sys.argv) > 2 and sys.argv[2] == "wide"   # config 5's cell kernels (scripts/counters_c5.sh)
acc = {}
for f in sorted(glob.glob(f"{root}/p*/c_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if wide:
            k = ("wide_cell_fwd" if "wide_cell_fwd_kernel" in k else
                 "wide_bwd_fused_l0" if "wide_bwd_fused_kernel" in k and ("Lb1E" in k or ", true" in k) else
                 "wide_bwd_fused" if "wide_bwd_fused_kernel" in k else None)
        else:
            k = "fwd" if "fcr_fwd_kernel" in k else "bwd" if "fcr_bwd_kernel" in k else None
        if k is None:
            continue
        acc.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {sum(v) / len(v):.4g}  (n={len(v)})")
