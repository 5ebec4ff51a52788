"""The committed profile summaries that bench.py's roofline reads (profiles/*_pmc.json) are well formed: the newest
default-benchmark summary gives the dominant kernel's HBM bytes per launch and the newest config-5 summary the
bytes of one backward pass (an empty summary would silently turn the bench line's `traffic` into null)."""
import glob
import json
import os
import re

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_newest_pmc_summaries_give_traffic():
    b, src = bench.pmc_traffic("fcr_bwd_kernel")
    f, _ = bench.pmc_traffic("fcr_fwd_kernel")
    assert b and f and b > 1e9 and f > 1e9, src
    c5, src5 = bench.pmc_traffic("bwd_pass", "_c5")
    assert c5 and c5 > 1e11, src5


def test_every_round_pmc_summary_has_its_kernels():
    for path in glob.glob(os.path.join(ROOT, "profiles", "round*_pmc.json")):
        d = json.load(open(path))
        keys = [k for k in d if not k.startswith("_")]
        assert keys, f"{os.path.basename(path)} holds no kernel"
        if re.search(r"_c5_pmc\.json$", path):
            assert d.get("bwd_pass", {}).get("hbm_bytes_corrected"), path


def test_config3_lines_read_their_own_pmc_summaries():
    for prec in ("f16", "fp32"):
        t, src = bench.pmc_traffic("fcr_bwd_kernel", f"_c3{prec}")
        assert t and t > 1e9 and f"c3{prec}" in src, src


def test_wide_cpu_baseline_times_the_lines_own_workload():
    """A config-5 line's cpu_baseline runs the CPU path at its own N and H (seeded weights), not config 2's."""
    r = bench.cpu_baseline(0.2, N=2, H=64)
    assert r["value"] > 0 and "N=2 H=64" in r["sample"], r["sample"]
    assert {x["batch"] for x in r["runs"]} == {15, 256}
    r50 = bench.cpu_baseline(0.2, N=2, H=50)
    assert "H=50" in r50["sample"] and {x["batch"] for x in r50["runs"]} == {15, 256, 4096}
