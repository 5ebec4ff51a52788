"""Data-parallel rollout across the GPUs of one node: one process per GPU, RCCL over xGMI.

The rollout shards trivially by trajectory (no cross-sample op before the batch mean,
Functions.py:1387-1463). Each rank runs the fused forward/backward on its B_local trajectories; the
only exchange is ONE all-reduce of the packed controller gradients (250 floats) plus the loss and the
shard size (two floats) per optimizer step — about 1 KB, latency-bound, so it is a single flat bucket,
not a bandwidth-tuned ring schedule. AdamW then runs identically on every rank (same reduced
gradients, same deterministic update), so no parameter broadcast is needed after the first sync.
"""
from __future__ import annotations

import warnings

import torch
import torch.distributed as dist


def shard_range(B_global: int, rank: int, world: int):
    """Contiguous shard [lo, hi) of the global batch owned by `rank` (equal shards when divisible)."""
    base, rem = divmod(B_global, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def broadcast_params(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Make every rank start from rank `src`'s controller weights."""
    for p in module.parameters():
        dist.broadcast(p.data, src=src, group=group)


class GradAllReduce:
    """Callable grad hook for ``NeuralNetwork.train_model(grad_sync=...)``.

    Each rank's loss is the mean over its B_local trajectories; the global loss is the mean over
    B_global = sum(B_local), so the global-mean gradient is sum_r (B_r / B_global) g_r.

    * ``hook(module, b_local, b_global)``: each rank scales by b_local / b_global before the SUM.
    * ``hook(module, b_local)`` (what ``train_model`` passes: the batch it just ran): b_local rides in the
      same buffer — [b_r g_r, b_r loss_r, b_r] is summed and divided by the summed b_r afterwards — so
      uneven shards and short last batches still give the global-mean gradient with ONE all-reduce.
    * ``hook(module)``: equal shards are assumed (1/world), with a one-time warning.

    Returns the global-mean loss when ``loss`` is given (every rank must then pass one), else None.

    Every rank packs the same buffer whatever its shard held: each trainable parameter's gradient (zeros
    where it has none) plus one has-gradient flag per parameter. A rank whose shard is EMPTY (more ranks
    than trajectories in a short last batch) therefore still joins the all-reduce with b_local = 0 and
    receives the others' gradients; a parameter no rank produced a gradient for (the idle ``fc_int``,
    Functions.py:279) keeps ``grad = None``, so AdamW skips it as it does in the reference.
    """

    def __init__(self, group=None):
        self.group = group
        self._warned = False
        self._flag_rows = {}   # has-gradient pattern -> its flag tensor on the device (built once, not per step)

    def _flags(self, pattern, like):
        key = (pattern, like.dtype, like.device)
        t = self._flag_rows.get(key)
        if t is None:
            t = torch.tensor([float(h) for h in pattern], dtype=like.dtype, device=like.device)
            self._flag_rows[key] = t
        return t

    def __call__(self, module: torch.nn.Module, b_local: int | None = None, b_global: int | None = None,
                 loss: torch.Tensor | None = None):
        params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            return loss
        world = dist.get_world_size(self.group)
        count = b_local is not None and not b_global
        if b_local is None and not self._warned:
            warnings.warn("GradAllReduce called without the shard size: assuming equal shards (1/world)")
            self._warned = True
        pieces = [p.grad.reshape(-1) if p.grad is not None else torch.zeros_like(p).reshape(-1) for p in params]
        pattern = tuple(p.grad is not None for p in params)
        pieces.append(self._flags(pattern, pieces[0]))
        if loss is not None:
            pieces.append(loss.detach().reshape(1).to(pieces[0].dtype))
        if count:
            pieces.append(pieces[0].new_ones(1))
        flat = torch.cat(pieces)
        nflag = len(params)
        off_flags = flat.numel() - nflag - (loss is not None) - count
        scale = float(b_local) if count else ((b_local / b_global) if b_local is not None else 1.0 / world)
        flat[:off_flags].mul_(scale)
        flat[off_flags + nflag:].mul_(scale)   # the loss and, in count mode, b_local itself
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        # a rank that ran the step produces gradients for the same parameters as every other such rank, so it
        # keeps its own pattern (no host sync); only a rank without any gradient reads the flags
        if any(pattern):
            flags = [float(h) for h in pattern]
        else:
            flags = flat[off_flags:off_flags + nflag].tolist()
        if count:
            flat = flat / flat[-1].clamp_min(1.0)   # sum of b_r (0 only if every shard was empty)
        off = 0
        for p, has in zip(params, flags):
            n = p.numel()
            if has > 0:
                if p.grad is None:
                    p.grad = torch.empty_like(p)
                p.grad.copy_(flat[off:off + n].view_as(p))
            off += n
        return flat[off_flags + nflag] if loss is not None else None
