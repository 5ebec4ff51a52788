"""Pure-Python restatement of the reference's sample producer (TEST INFRASTRUCTURE ONLY).

* ``SequenceDataset.__getitem__``   Functions.py:109-132 -> :func:`sequence_item`
* ``Data.get_individual_dataset``   Functions.py:479-516 + ``ConcatDataset`` (UL/Main.py:275-279)
                                     -> :func:`concat_item`

PARITY STATUS: the restatement follows the reference's indexing line by line (left padding with the
trajectory's first row for i < lookback-1, target y[i+1] clamped to the last row, IndexError at
i >= len); the reference has no tests of its own for it, and the GPU gather is held bit-exact to it.
"""
from __future__ import annotations

import numpy as np


def sequence_item(X, Y, Z, i, lookback=10):
    """One trajectory's (x, y, z) for local row i, Functions.py:111-132."""
    L = X.shape[0]
    if i >= L:
        raise IndexError(i)
    x = X[i]
    if i >= lookback - 1:
        z = Z[i - lookback + 1:i + 1]
    else:
        z = np.concatenate([np.repeat(Z[:1], lookback - i - 1, axis=0), Z[:i + 1]], axis=0)
    y = Y[i + 1] if i < L - 1 else Y[-1]
    return x, y, z


def concat_item(X, Y, Z, g, traj_len, lookback=10):
    """ConcatDataset over trajectories of traj_len rows: global index g -> (trajectory, local row)."""
    if g < 0 or g >= X.shape[0]:
        raise IndexError(g)
    k, i = divmod(g, traj_len)
    s = slice(k * traj_len, (k + 1) * traj_len)
    return sequence_item(X[s], Y[s], Z[s], i, lookback)
