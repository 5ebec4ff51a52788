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
