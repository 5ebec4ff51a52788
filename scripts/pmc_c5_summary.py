"""Config-5 PMC summary (scripts/profile.sh TAG c5|c5max): HBM bytes per launch of the main H = 256 kernels, and the
HBM bytes of one whole backward pass (every dispatch from its first wide_head_kernel to the ctrl_grad_kernel after it),
FETCH_SIZE / WRITE_SIZE in separate passes with the gfx950 correction (2 x FETCH + WRITE, MI355X_MICROARCH.md).
    python scripts/pmc_c5_summary.py TAG DIR  ->  profiles/TAG_c5_pmc.json, profiles/TAG_c5_kernel_stats.csv"""
import csv
import glob
import json
import shutil
import sys

tag, root = sys.argv[1], sys.argv[2]
KERNELS = ("wide_cell_fwd_kernel", "wide_bwd_fused_kernel", "wide_head_kernel")
INST = ("SQ_INSTS_VALU_MFMA_F16", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY",
        "SQ_LDS_BANK_CONFLICT", "GRBM_GUI_ACTIVE")


def dispatches(kind, counter):
    f = glob.glob(f"{root}/{kind}/**/*counter_collection.csv", recursive=True)
    by = {}
    for r in (csv.DictReader(open(f[0])) if f else []):
        if r["Counter_Name"] != counter:
            continue
        k = int(r["Dispatch_Id"])
        name, v = by.get(k, (r["Kernel_Name"], 0.0))
        by[k] = (name, v + float(r["Counter_Value"]))
    return [by[k] for k in sorted(by)]


out = {}
passes = {}
for kind, cnt in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    ds = dispatches(kind, cnt)
    for name in KERNELS:
        vals = [v for n, v in ds if name in n]
        if vals:
            out.setdefault(name, {})[cnt + "_KB_per_launch"] = sum(vals) / len(vals)
            out[name]["launches"] = len(vals)
    # backward passes: the first wide_head_kernel after a forward's loss_reduce_kernel .. the next ctrl_grad_kernel
    # (inclusive); the last one profiled counts
    tot, on, last, fwd_done = 0.0, False, None, False
    for n, v in ds:
        if "loss_reduce_kernel" in n:
            fwd_done = True
        if fwd_done and "wide_head_kernel" in n and not on:
            on, tot, fwd_done = True, 0.0, False
        if on:
            tot += v
        if on and "ctrl_grad_kernel" in n:
            on, last = False, tot
    passes[cnt] = last
for cnt in INST:   # instruction / wait counters of the same kernels (one pass; per launch, summed over the device)
    for name in KERNELS:
        vals = [v for n, v in dispatches("inst", cnt) if name in n]
        if vals:
            out.setdefault(name, {})[cnt + "_per_launch"] = sum(vals) / len(vals)
for name, d in out.items():
    if "FETCH_SIZE_KB_per_launch" in d and "WRITE_SIZE_KB_per_launch" in d:
        d["hbm_bytes_corrected"] = (2 * d["FETCH_SIZE_KB_per_launch"] + d["WRITE_SIZE_KB_per_launch"]) * 1024
if passes.get("FETCH_SIZE") is not None and passes.get("WRITE_SIZE") is not None:
    out["bwd_pass"] = {"FETCH_SIZE_KB": passes["FETCH_SIZE"], "WRITE_SIZE_KB": passes["WRITE_SIZE"],
                       "hbm_bytes_corrected": (2 * passes["FETCH_SIZE"] + passes["WRITE_SIZE"]) * 1024}
out["_note"] = ("rocprofv3 PMC passes of bench.py --hidden 256 --horizon 25 --batch 65536 (config 5), KB; "
                "hbm_bytes_corrected = 2*FETCH + WRITE (gfx950); SQ_* / GRBM_* per launch from one more pass (SQ_WAVE_CYCLES and "
                "SQ_WAIT_INST_ANY in quad-cycles, MI355X_MICROARCH.md). bwd_pass = every dispatch of the last profiled "
                "backward pass, its first wide_head_kernel .. ctrl_grad_kernel.")
stats = glob.glob(f"{root}/trace/**/*kernel_stats.csv", recursive=True)
if stats:
    shutil.copy(stats[0], f"profiles/{tag}_c5_kernel_stats.csv")
json.dump(out, open(f"profiles/{tag}_c5_pmc.json", "w"), indent=1)
print(json.dumps(out, indent=1))
