"""CPU: the backward weight image layout (fcr_img.h) — every recompute row read and transposed read
fetches the intended weight, with lane base + instruction-constant addressing and no LDS bank conflict."""
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "scripts"))
import img_layout_check  # noqa: E402


@pytest.mark.parametrize("HS", [4, 8, 13])
@pytest.mark.parametrize("layer", [0, 1])
def test_image_layout_conflict_free(HS, layer):
    U, tile, fconf, tconf = img_layout_check.check(HS, layer)
    assert fconf == 0 and tconf == 0
    assert tile * 8 * HS <= 16 * HS * U * 8 * 1.05   # stagger costs <= 5 % over packed rows
