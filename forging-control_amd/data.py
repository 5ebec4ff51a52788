"""Device-resident training samples.

The reference feeds ``train_model`` through ``DataLoader(ConcatDataset([SequenceDataset(traj) ...]),
batch_size, shuffle)`` (UL/Main.py:270-304), building every sample in Python
(``SequenceDataset.__getitem__``, Functions.py:109-132) and copying each batch to the device
(Functions.py:637). :class:`SequenceWindows` keeps the concatenated tables in HBM and gathers a whole
batch with one HIP launch (``fcr_window_gather``, forging-control_amd/csrc/fcr_window.h);
:class:`DeviceLoader` is the DataLoader over it (same batch order semantics: a fresh permutation per
epoch when shuffling, the index order otherwise).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native


def _dev_table(t, name, device):
    t = torch.as_tensor(t)
    if t.dim() == 1:
        t = t.unsqueeze(1)
    if t.dim() != 2:
        raise ValueError(f"{name} must be (rows, features), got {tuple(t.shape)}")
    return t.to(device=device, dtype=torch.float32).contiguous()


class SequenceWindows:
    """ConcatDataset of SequenceDataset (Functions.py:92-132) over trajectories of ``traj_len`` rows.

    ``X`` (rows, 3) static features, ``Y`` (rows, 1) target, ``Z`` (rows, 5) recurrent features; item g
    is ``(x, y, z)`` exactly as ``ConcatDataset.__getitem__(g)`` returns it (z of shape (lookback, 5))."""

    def __init__(self, X, Y, Z, traj_len: int, lookback: int = 10, device="cuda"):
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError(f"SequenceWindows lives on a ROCm device (got {device}); there is no CPU path")
        self.X, self.Y, self.Z = (_dev_table(t, n, device) for t, n in ((X, "X"), (Y, "Y"), (Z, "Z")))
        rows = self.X.shape[0]
        if self.Y.shape[0] != rows or self.Z.shape[0] != rows:
            raise ValueError("X, Y and Z must have the same number of rows")
        if traj_len < 1 or rows % traj_len:
            raise ValueError(f"rows={rows} must be a positive multiple of traj_len={traj_len}")
        self.traj_len, self.lookback, self.device = int(traj_len), int(lookback), device
        self._tables = _native.FcrWindows(rows, self.traj_len, self.lookback, self.X.shape[1], self.Y.shape[1],
                                          self.Z.shape[1], self.X.data_ptr(), self.Y.data_ptr(), self.Z.data_ptr())
        self._bad = torch.zeros(1, dtype=torch.int32, device=device)

    @classmethod
    def from_dataframe(cls, df, target, features, recurrent_features, t_traj: int, lookback: int = 10,
                       device="cuda"):
        """Data.get_individual_dataset (Functions.py:479-516) + ConcatDataset: whole trajectories of
        ``t_traj`` rows (a trailing partial trajectory is dropped, as the reference's range does)."""
        n = (len(df) // t_traj) * t_traj
        d = df.iloc[:n]
        return cls(np.asarray(d[features].values, np.float32), np.asarray(d[target].values, np.float32),
                   np.asarray(d[recurrent_features].values, np.float32), t_traj, lookback, device)

    def __len__(self):
        return self.X.shape[0]

    def gather(self, idx, check: bool = True):
        """(x (B,nx), y (B,ny), z (B,lookback,nz)) for global indices idx (B,). ``check`` raises
        IndexError for indices outside [0, len) (one device->host read of the kernel's counter)."""
        idx = torch.as_tensor(idx, device=self.device).to(torch.int64).reshape(-1).contiguous()
        B = idx.shape[0]
        f32 = dict(dtype=torch.float32, device=self.device)
        x = torch.empty(B, self.X.shape[1], **f32)
        y = torch.empty(B, self.Y.shape[1], **f32)
        z = torch.empty(B, self.lookback, self.Z.shape[1], **f32)
        lib = _native.load()
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        _native.check(lib.fcr_window_gather(ctypes.byref(self._tables), B, p(idx), p(x), p(y), p(z), p(self._bad),
                                            ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
                      "fcr_window_gather")
        if check and int(self._bad.item()):
            raise IndexError(f"{int(self._bad.item())} index(es) outside [0, {len(self)})")
        return x, y, z

    def __getitem__(self, i):
        x, y, z = self.gather([i])
        return x[0], y[0], z[0]


class DeviceLoader:
    """DataLoader(windows or Subset(windows, indices), batch_size, shuffle) yielding device batches.

    ``indices`` plays torch.utils.data.Subset (UL/Main.py:282-291 resamples every N-th sample)."""

    def __init__(self, windows: SequenceWindows, batch_size: int, shuffle: bool = False, indices=None,
                 generator: torch.Generator | None = None, check: bool = False):
        self.w, self.batch_size, self.shuffle, self.check = windows, int(batch_size), bool(shuffle), check
        base = torch.arange(len(windows)) if indices is None else torch.as_tensor(indices, dtype=torch.int64)
        self.indices = base.to(windows.device)
        self.generator = generator

    def __len__(self):
        return (self.indices.numel() + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        order = self.indices
        if self.shuffle:
            perm = torch.randperm(order.numel(), generator=self.generator).to(order.device)
            order = order[perm]
        for s in range(0, order.numel(), self.batch_size):
            yield self.w.gather(order[s:s + self.batch_size], check=self.check)
