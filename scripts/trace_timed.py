"""Per-kernel durations of the TIMED steps only, from a rocprofv3 kernel trace of `bench.py --steps K --warmup W`.

The kernel statistics (`*_kernel_stats.csv`) average every dispatch of a kernel, including the W warm-up steps and
the grad check's extra launch after the timed region; the bench line's `ms_per_step` covers the K timed steps only.
This takes the rollout kernels' dispatches in launch order, drops the first W and keeps the next K, so their mean
durations and the bench line's step time describe the same launches.

    python scripts/trace_timed.py TRACE_CSV W K  [OUT_JSON]
"""
import csv
import json
import sys

path, W, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = [r for r in csv.DictReader(open(path))]
out = {}
for key, pat in (("fwd", "fcr_fwd_kernel"), ("bwd", "fcr_bwd_kernel")):
    d = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if pat in r["Kernel_Name"])
    timed = d[W:W + K]
    if len(timed) < K:
        sys.exit(f"{pat}: {len(d)} dispatches, need {W + K}")
    ms = [(e - s) / 1e6 for s, e in timed]
    out[key] = {"timed_dispatches": K, "mean_ms": sum(ms) / K, "min_ms": min(ms), "max_ms": max(ms),
                "all_dispatches": len(d), "all_mean_ms": sum((e - s) / 1e6 for s, e in d) / len(d)}
out["fwd_plus_bwd_ms"] = out["fwd"]["mean_ms"] + out["bwd"]["mean_ms"]
out["_note"] = f"{path}: dispatches {W}..{W + K - 1} of each rollout kernel (the timed steps of bench.py --warmup {W} --steps {K})"
print(json.dumps(out, indent=1))
if len(sys.argv) > 4:
    json.dump(out, open(sys.argv[4], "w"), indent=1)
