"""Summarise a profile (scripts/profile.sh) into profiles/<tag>_pmc.json and profiles/<tag>_kernel_stats.csv: HBM
bytes per launch (FETCH_SIZE / WRITE_SIZE passes, gfx950 correction), MFMA / VALU / LDS instructions per launch and
per wave-cell, and the clock each kernel ran at.
    python scripts/pmc_summary.py TAG DIR [bench.py --batch/--horizon/--precision arguments]"""
import argparse
import csv
import glob
import json
import shutil

ap = argparse.ArgumentParser()
ap.add_argument("tag")
ap.add_argument("root")
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--horizon", type=int, default=10)
ap.add_argument("--precision", default="fp32")
args = ap.parse_args()
tag, root = args.tag, args.root
KERNELS = ("fcr_fwd_kernel", "fcr_bwd_kernel")
B, N, L, LAYERS, TILE = args.batch, args.horizon, 10, 3, 16
WAVES = (B + TILE - 1) // TILE


def rows(kind):
    f = glob.glob(f"{root}/{kind}/**/*counter_collection.csv", recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def per_launch(rs, name, counter):
    # one row per (dispatch, counter); values are summed over the dispatch's XCDs / SEs by rocprofv3
    by = {}
    for r in rs:
        if name in r["Kernel_Name"] and r["Counter_Name"] == counter:
            by[r.get("Dispatch_Id", len(by))] = by.get(r.get("Dispatch_Id", len(by)), 0.0) + float(r["Counter_Value"])
    return (sum(by.values()) / len(by), len(by)) if by else (None, 0)


out = {}
for name in KERNELS:
    d = {}
    for kind, cnt in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        v, n = per_launch(rows(kind), name, cnt)
        d[cnt + "_KB_per_launch"] = v
        d["launches"] = n
    if d["FETCH_SIZE_KB_per_launch"] is not None and d["WRITE_SIZE_KB_per_launch"] is not None:
        d["hbm_bytes_raw"] = (d["FETCH_SIZE_KB_per_launch"] + d["WRITE_SIZE_KB_per_launch"]) * 1024
        d["hbm_bytes_corrected"] = (2 * d["FETCH_SIZE_KB_per_launch"] + d["WRITE_SIZE_KB_per_launch"]) * 1024
    ins = rows("inst")
    for cnt in ("SQ_INSTS_VALU_MFMA_F16", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_WAVES", "GRBM_GUI_ACTIVE"):
        d[cnt + "_per_launch"] = per_launch(ins, name, cnt)[0]
    wt = rows("wait")   # the issue / wait split (MI355X_MICROARCH.md PMC: the three SQ_*ANY buckets are disjoint)
    for cnt in ("SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VMEM"):
        d[cnt + "_per_launch"] = per_launch(wt, name, cnt)[0]
    wc = d["SQ_WAVE_CYCLES_per_launch"]
    if wc:
        for cnt, key in (("SQ_ACTIVE_INST_ANY", "issue"), ("SQ_ACTIVE_INST_VALU", "issue_valu"),
                         ("SQ_WAIT_INST_ANY", "issue_wait"), ("SQ_WAIT_ANY", "waitcnt_barrier")):
            d["share_" + key] = d[cnt + "_per_launch"] / wc
        # two waves per SIMD (8-wave workgroups, one per CU): the SIMD's vector issue busy = 2 x a wave's share
        d["simd_valu_issue_busy"] = 2 * d["share_issue_valu"]
    g = per_launch(wt, name, "GRBM_GUI_ACTIVE")[0]
    if g and d.get("SQ_VALU_MFMA_BUSY_CYCLES_per_launch"):
        # cycles the matrix pipe of a SIMD is busy over the kernel's cycles (GRBM_GUI_ACTIVE sums the 8 XCDs)
        d["simd_mfma_busy"] = d["SQ_VALU_MFMA_BUSY_CYCLES_per_launch"] / (1024 * g / 8)
    m = d["SQ_INSTS_VALU_MFMA_F16_per_launch"]
    if m:
        d["mfma_per_wave_cell"] = m / (WAVES * N * L * LAYERS)
        d["valu_non_mfma_per_wave_cell"] = (d["SQ_INSTS_VALU_per_launch"] - m) / (WAVES * N * L * LAYERS)
        d["mfma_flop_per_launch"] = m * 16 * 16 * 32 * 2
    out[name] = d

stats = glob.glob(f"{root}/trace/**/*kernel_stats.csv", recursive=True)
if stats:
    shutil.copy(stats[0], f"profiles/{tag}_kernel_stats.csv")
    for r in csv.DictReader(open(stats[0])):
        for name in KERNELS:
            if name in r["Name"]:
                out[name]["rocprof_avg_ms"] = float(r["AverageNs"]) / 1e6
                out[name]["rocprof_calls"] = int(r["Calls"])
for name in KERNELS:
    d = out[name]
    if d.get("GRBM_GUI_ACTIVE_per_launch") and d.get("rocprof_avg_ms"):
        # MI355X_MICROARCH.md DVFS: clock ~ GRBM_GUI_ACTIVE / 8 XCDs / kernel time
        d["clock_ghz_est"] = d["GRBM_GUI_ACTIVE_per_launch"] / 8 / (d["rocprof_avg_ms"] * 1e-3) / 1e9
    if d.get("hbm_bytes_corrected") and d.get("rocprof_avg_ms"):
        d["hbm_tb_per_s"] = d["hbm_bytes_corrected"] / (d["rocprof_avg_ms"] * 1e-3) / 1e12
    if d.get("mfma_flop_per_launch") and d.get("rocprof_avg_ms"):
        d["mfma_tflops_executed"] = d["mfma_flop_per_launch"] / (d["rocprof_avg_ms"] * 1e-3) / 1e12
out["_note"] = (f"rocprofv3 PMC passes of bench.py B={B} N={N} H=50 {args.precision} (scripts/profile.sh): FETCH_SIZE and "
                "WRITE_SIZE in separate passes, KB; hbm_bytes_corrected = 2*FETCH (gfx950 reports half of wide "
                "coalesced reads, MI355X_MICROARCH.md HBM) + WRITE. Instruction counts are wave-instructions per "
                "launch; per wave-cell = / (B/16 waves * N windows * 10 steps * 3 layers). share_* = SQ_ACTIVE_INST_ANY / "
                "SQ_ACTIVE_INST_VALU / SQ_WAIT_INST_ANY / SQ_WAIT_ANY over SQ_WAVE_CYCLES (per wave); simd_valu_issue_busy = "
                "2 waves per SIMD x share_issue_valu; simd_mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x "
                "GRBM_GUI_ACTIVE / 8).")
json.dump(out, open(f"profiles/{tag}_pmc.json", "w"), indent=1)
print(json.dumps(out, indent=1))
