"""Summarise scripts/counters.sh passes: per kernel, mean counter value per launch."""
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ctr"
acc = {}
for f in sorted(glob.glob(f"{root}/p*/c_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        k = "fwd" if "fcr_fwd_kernel" in k else "bwd" if "fcr_bwd_kernel" in k else None
        if k is None:
            continue
        acc.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {sum(v) / len(v):.4g}  (n={len(v)})")
