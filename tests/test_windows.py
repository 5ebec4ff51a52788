"""Device window gather vs the restated SequenceDataset/ConcatDataset."""
import ctypes
import importlib

import numpy as np
import pytest
import torch

from oracle.windows_ref import concat_item, sequence_item

fca = importlib.import_module("forging-control_amd")


def _tables(n_traj, traj_len, seed=0, nx=3, ny=1, nz=5):
    rng = np.random.default_rng(seed)
    rows = n_traj * traj_len
    return (rng.standard_normal((rows, nx)).astype(np.float32), rng.standard_normal((rows, ny)).astype(np.float32),
            rng.standard_normal((rows, nz)).astype(np.float32))


def test_oracle_padding_and_target_rules():
    X, Y, Z = _tables(1, 12)
    x, y, z = sequence_item(X, Y, Z, 0)
    assert np.array_equal(z, np.repeat(Z[:1], 10, axis=0)) and np.array_equal(y, Y[1]) and np.array_equal(x, X[0])
    _, _, z = sequence_item(X, Y, Z, 3)          # 6 padding rows, then rows 0..3 (Functions.py:118-121)
    assert np.array_equal(z[:6], np.repeat(Z[:1], 6, axis=0)) and np.array_equal(z[6:], Z[:4])
    _, _, z = sequence_item(X, Y, Z, 9)          # first full window
    assert np.array_equal(z, Z[:10])
    _, y, z = sequence_item(X, Y, Z, 11)         # last row: target clamps to y[-1] (:124-127)
    assert np.array_equal(y, Y[-1]) and np.array_equal(z, Z[2:12])
    with pytest.raises(IndexError):
        sequence_item(X, Y, Z, 12)


def test_oracle_concat_never_crosses_trajectories():
    X, Y, Z = _tables(3, 15)
    _, y, z = concat_item(X, Y, Z, 15, 15)       # first row of trajectory 1: padded with ITS first row
    assert np.array_equal(z, np.repeat(Z[15:16], 10, axis=0)) and np.array_equal(y, Y[16])
    _, y, _ = concat_item(X, Y, Z, 29, 15)       # last row of trajectory 1: target stays inside it
    assert np.array_equal(y, Y[29])


def test_windows_refuse_cpu():
    X, Y, Z = _tables(1, 10)
    with pytest.raises(RuntimeError, match="ROCm device"):
        fca.SequenceWindows(X, Y, Z, 10, device="cpu")


@pytest.mark.parametrize("kw,msg", [(dict(rows=25, traj_len=10), "multiple"), (dict(lookback=0), "lookback"),
                                    (dict(nz=-1), "feature"), (dict(), "NULL")])
def test_abi_rejects_bad_tables_before_any_device_call(kw, msg):
    lib = fca._native.load()
    t = dict(rows=20, traj_len=10, lookback=10, nx=3, ny=1, nz=5)
    t.update(kw)
    tab = fca._native.FcrWindows(t["rows"], t["traj_len"], t["lookback"], t["nx"], t["ny"], t["nz"], None, None, None)
    assert lib.fcr_window_gather(ctypes.byref(tab), 4, None, None, None, None, None, None) == -1
    assert msg in lib.fcr_last_error().decode()


# ------------------------------------------------------------------------------------------------ GPU

def _oracle_batch(X, Y, Z, idx, traj_len, lookback):
    items = [concat_item(X, Y, Z, int(g), traj_len, lookback) for g in idx]
    return [np.stack([it[k] for it in items]) for k in range(3)]


@pytest.mark.gpu
@pytest.mark.parametrize("n_traj,traj_len,lookback", [(3, 37, 10), (1, 5, 10), (4, 20, 1), (2, 150, 10), (5, 9, 25)])
def test_gpu_gather_bit_exact(n_traj, traj_len, lookback):
    X, Y, Z = _tables(n_traj, traj_len, seed=traj_len)
    w = fca.SequenceWindows(X, Y, Z, traj_len, lookback)
    idx = np.random.default_rng(1).permutation(len(w))
    got = [t.cpu().numpy() for t in w.gather(torch.tensor(idx))]
    ref = _oracle_batch(X, Y, Z, idx, traj_len, lookback)
    for g, r in zip(got, ref):
        assert g.shape == r.shape and np.array_equal(g, r)


@pytest.mark.gpu
def test_gpu_gather_index_errors_and_empty_batch():
    X, Y, Z = _tables(2, 10)
    w = fca.SequenceWindows(X, Y, Z, 10)
    with pytest.raises(IndexError):
        w.gather([0, 20])
    with pytest.raises(IndexError):
        w.gather([-1])
    x, y, z = w.gather(torch.zeros(0, dtype=torch.int64))
    assert x.shape == (0, 3) and y.shape == (0, 1) and z.shape == (0, 10, 5)
    xi, yi, zi = w[13]
    rx, ry, rz = concat_item(X, Y, Z, 13, 10)
    assert np.array_equal(xi.cpu().numpy(), rx) and np.array_equal(zi.cpu().numpy(), rz)


@pytest.mark.gpu
def test_gpu_device_loader_epoch_semantics():
    X, Y, Z = _tables(4, 30, seed=3)
    w = fca.SequenceWindows(X, Y, Z, 30)
    seen = []
    for x, y, z in fca.DeviceLoader(w, 15, shuffle=True, generator=torch.Generator().manual_seed(0)):
        assert x.shape[0] <= 15
        seen.append(x.cpu().numpy())
    got = np.concatenate(seen)
    assert got.shape == X.shape and np.array_equal(np.sort(got, axis=0), np.sort(X, axis=0))
    sub = list(range(0, len(w), 10))                  # UL/Main.py:282-291 resampling, in order
    xs = np.concatenate([b[0].cpu().numpy() for b in fca.DeviceLoader(w, 4, indices=sub)])
    assert np.array_equal(xs, X[sub])
