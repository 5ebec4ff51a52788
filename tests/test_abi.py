"""CPU: the C-ABI library loads, exports exactly what include/fcr.h declares, and validates dims
(no compute calls: there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

import forging_control_amd as fca
from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "fcr.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(fcr_\w+)\s*\(", text, re.M)))


def test_header_declares_every_exported_entry_point():
    assert declared_symbols() == sorted(fca._native.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = fca._native.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", fca._native.LIB_PATH], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l and l.split()[-1].startswith("fcr_")}
    assert exported == set(declared_symbols())


def test_library_targets_gfx950():
    blob = open(fca._native.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_abi_version():
    assert fca._native.load().fcr_abi_version() == fca._native.ABI_VERSION


def dims(**kw):
    base = dict(B=65536, N=10, H=50, layers=3, ctrl_hidden=50, alpha=20.0, precision=0)
    base.update(kw)
    return fca.rollout.make_dims(base["B"], base["N"], base["H"], base["layers"], base["ctrl_hidden"], base["alpha"],
                                 precision=base["precision"])


def test_workspace_size_scales_with_batch_and_backward():
    small = fca._native.workspace_bytes(dims(B=128), True)    # 8 waves of 16 trajectories (one forward workgroup)
    big = fca._native.workspace_bytes(dims(B=65536), True)    # 4096 waves
    fwd_only = fca._native.workspace_bytes(dims(B=65536), False)
    assert 0.97 * 512 * small < big < 1.01 * 512 * small   # fixed fragment blocks are the slack
    # h and c of 10 windows x 30 cells x 52 units fp32 per trajectory (the backward recomputes the rest)
    assert big > 65536 * 10 * 30 * 52 * 2 * 4
    assert fwd_only < big / 2          # forward-only keeps just the h slab (inter-layer hand-off)


@pytest.mark.parametrize("kw,code", [
    (dict(B=0), -1), (dict(N=0), -1), (dict(H=4096), -4), (dict(H=0), -4), (dict(layers=2), -4), (dict(ctrl_hidden=80), -4),
    (dict(precision=3), -1), (dict(precision=1, H=64), -4), (dict(precision=2), -4),
])
def test_invalid_dims_rejected_with_message(kw, code):
    lib = fca._native.load()
    out = ctypes.c_size_t(0)
    d = dims(**kw)
    rc = lib.fcr_workspace_size(ctypes.byref(d), None, 1, ctypes.byref(out))
    assert rc == code
    assert lib.fcr_last_error().decode()


def test_null_pointers_rejected_before_any_device_call():
    lib = fca._native.load()
    d = dims(B=16)
    w = fca._native.FcrWeights()
    rc = lib.fcr_forward(ctypes.byref(d), None, ctypes.byref(w), *([None] * 10), 1, None, 0, None)
    assert rc == -1 and "NULL" in lib.fcr_last_error().decode()
    rc = lib.fcr_backward(ctypes.byref(d), None, *([None] * 8), None, 0, None)
    assert rc == -1


def test_fnn_entry_points_validate_before_any_device_call():
    lib = fca._native.load()
    out = ctypes.c_size_t(0)
    assert lib.fcr_fnn_workspace_size(65536, 50, ctypes.byref(out)) == 0
    assert out.value == 256 * 50 * 5 * 4          # one partial record per 256-sample block
    assert lib.fcr_fnn_workspace_size(65536, 65, ctypes.byref(out)) == -1
    assert lib.fcr_fnn_forward(16, 4, 50, *([None] * 5), None) == -4      # in_dim != 3
    assert "in_dim" in lib.fcr_last_error().decode()
    assert lib.fcr_fnn_forward(16, 3, 80, *([None] * 5), None) == -4      # hidden > 64
    assert lib.fcr_fnn_forward(16, 3, 50, *([None] * 5), None) == -1      # NULL
    assert lib.fcr_fnn_forward(0, 3, 50, *([None] * 5), None) == 0        # empty batch: no launch
    assert lib.fcr_fnn_backward(-1, 3, 50, *([None] * 10), 0, None) == -1
    assert lib.fcr_fnn_backward(16, 3, 50, *([None] * 10), 0, None) == -1


def test_fnn_model_on_cpu_is_the_torch_module():
    """CPU tensors never reach the HIP path (it is selected for ROCm tensors of the reference's shape)."""
    import torch
    m = fca.FNNModel(3, 50, 1, 1)
    x = torch.randn(7, 3)
    from forging_control_amd.controller import hip_shape_ok
    assert not hip_shape_ok(m, x)
    ref = torch.nn.functional.hardtanh(m.fc_out(torch.relu(m.fc_inp(x))))
    assert torch.equal(m(x), ref)


def test_process_defaults_have_read_only_getters():
    """fcr_set_small_batch_limit / fcr_set_wide_keep_budget set the process-wide DEFAULTS of the per-call options;
    the getters read them without changing them (reading by set-and-restore let another thread see 0)."""
    import threading
    n = fca._native
    prev = n.set_small_batch_limit(77)
    try:
        assert n.small_batch_limit() == 77 and n.small_batch_limit() == 77
        seen = {}
        th = threading.Thread(target=lambda: seen.setdefault("other", n.small_batch_limit()))
        th.start()
        th.join()
        assert seen["other"] == 77
        assert n.set_small_batch_limit(-5) == 77 and n.small_batch_limit() == 0   # negative clamps to 0 = never
    finally:
        n.set_small_batch_limit(prev)
    kb = n.wide_keep_budget()
    assert kb == -1   # the library's policy
    assert n.set_wide_keep_budget(123) == -1 and n.wide_keep_budget() == 123
    n.set_wide_keep_budget(kb)


def test_options_and_workspace_queries_validate_on_the_host():
    """Per-call options (fcr_options) reach fcr_workspace_size: an H > 52 backward workspace grows by whole kept
    windows with the call's budget, and fcr_wide_kept_windows reports the count a workspace holds."""
    n = fca._native
    d = dims(B=64, N=4, H=64)
    floor = n.workspace_bytes(d, True, n.make_options(wide_keep_budget=0))
    one = n.workspace_bytes(d, True, n.make_options(wide_keep_budget=4 * 3 * 10 * 64 * 5 * 64 + 4096))
    every = n.workspace_bytes(d, True, n.make_options(wide_keep_budget=1 << 40))
    assert floor < one < every
    assert [n.kept_windows(d, b) for b in (floor, one, every)] == [0, 1, 4]
    assert n.kept_windows(dims(B=64), 1 << 30) == 0                 # H <= 52: no kept windows
    with pytest.raises(ValueError):
        n.make_options(wide_keep_budget=-7)
    with pytest.raises(ValueError):
        n.make_options(small_batch_limit=-1)
    o = n.make_options()
    assert (o.small_batch_limit, o.wide_keep_budget, o.kernels) == (n.OPT_INHERIT, n.OPT_INHERIT, 0)
    assert n.make_options(wide_keep_budget="auto").wide_keep_budget == n.KEEP_AUTO


def test_pipe_defaults_have_read_only_getters():
    """fcr_set_small_pipe_limit / fcr_set_small_pipe_sets (the layer-pipelined small-batch geometry, csrc/fcr_pipe.h):
    setters return the previous value, negatives clamp to 0 (= never / automatic), the window-set cap clamps to the
    forward's maximum of 4, and the getters read without changing anything."""
    n = fca._native
    prev_limit, prev_sets = n.small_pipe_limit(), n.small_pipe_sets()
    try:
        assert n.set_small_pipe_limit(33) == prev_limit and n.small_pipe_limit() == 33 and n.small_pipe_limit() == 33
        assert n.set_small_pipe_limit(-1) == 33 and n.small_pipe_limit() == 0
        assert n.set_small_pipe_sets(9) == prev_sets and n.small_pipe_sets() == 4
        assert n.set_small_pipe_sets(-3) == 4 and n.small_pipe_sets() == 0
    finally:
        n.set_small_pipe_limit(prev_limit)
        n.set_small_pipe_sets(prev_sets)
    assert (n.small_pipe_limit(), n.small_pipe_sets()) == (prev_limit, prev_sets)


@pytest.mark.parametrize("B,N,H", [(2**31 - 1, 10, 50), (65536, 2**31 - 1, 50), (2**31 - 1, 10, 2048), (2**30, 1000, 256)])
def test_workspace_size_refuses_overflowing_dims(B, N, H):
    """Sizes whose trajectory-step count or workspace would overflow are refused with a message, never wrapped."""
    lib = fca._native.load()
    out = ctypes.c_size_t(0)
    rc = lib.fcr_workspace_size(ctypes.byref(dims(B=B, N=N, H=H)), None, 1, ctypes.byref(out))
    assert rc == -1 and out.value == 0
    assert "too large" in lib.fcr_last_error().decode()
