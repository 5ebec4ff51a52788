"""Whole training steps replayed from HIP graphs — the launch-bound small-batch regime.

The reference trains the controller with B = 15 trajectories per batch (UL/Main.py:283-309) and the
surrogate with B = 256 windows (Model_NN/Main.py:218-242). At those sizes a step —
``zero_grad(); output = model(X); loss = loss_function(...); loss.backward(); optimizer.step()``
(UL/Functions.py:640-658, Model_NN/Functions.py:520-569) — is microseconds of kernel work behind tens of
host-side launches (ctypes calls, autograd, the optimizer's foreach kernels). :class:`CapturedStep`
records the whole step once into a HIP graph (``torch.cuda.CUDAGraph`` = hipGraph on ROCm) and replays
it per batch: one graph launch instead of the launch sequence, the same kernels, the same results.

Only the batch tensors change between replays: they are copied into the graph's static inputs. The
captured region is exactly the eager step, so every kernel — the fused rollout, the controller, the
surrogate's cells and GEMMs, AdamW — is the HIP path it is without the graph. Batches of another shape
(the loader's last, short batch) run the same step eagerly. With a ``grad_sync`` hook (data parallelism)
the step is two graphs — forward + backward, then the optimizer — with the RCCL all-reduce issued
eagerly between them.

The optimizer must keep its step counter on the device (``capturable=True`` for torch's Adam/AdamW);
:class:`CapturedStep` switches a fresh or CPU-stepped optimizer over. That evaluates AdamW's bias
corrections in fp32 on the device instead of fp64 on the host (parameter differences ~1e-7 relative).
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch


def _make_capturable(optimizer: torch.optim.Optimizer) -> None:
    for group in optimizer.param_groups:
        if group.get("capturable", True):   # no flag (e.g. SGD): no host-side step state to move
            continue
        group["capturable"] = True
        for p in group["params"]:
            st = optimizer.state.get(p)
            if st and "step" in st and st["step"].device != p.device:
                st["step"] = st["step"].to(device=p.device, dtype=torch.float32)


class CapturedStep:
    """``step(*batch)`` = zero_grad -> ``body(*batch)`` -> [``grad_sync(*batch)``] -> ``optimizer.step()``.

    ``body`` runs the forward AND calls ``backward()`` itself; it returns a tuple of tensors (loss and
    whatever else the caller keeps). The first ``warmup`` calls run eagerly on a side stream (they are
    real training steps: library handles, optimizer state and the allocator settle); the next call of
    the same batch shape captures the step and every later one replays it. Returned tensors of a
    replayed step are the graph's static outputs — overwritten by the next call, so clone what you keep.
    """

    def __init__(self, params: Sequence[torch.Tensor], optimizer: torch.optim.Optimizer,
                 body: Callable[..., tuple], grad_sync: Callable[..., None] | None = None, warmup: int = 2):
        self.params = list(params)
        self.optimizer = optimizer
        self.body = body
        self.grad_sync = grad_sync
        self.warmup = max(int(warmup), 1)   # AdamW's state must exist before the capture
        self.eager_steps = 0
        self.replays = 0
        self._key = None
        self._g_fb = self._g_opt = None
        _make_capturable(optimizer)

    @staticmethod
    def _shape_key(batch):
        return tuple((tuple(t.shape), t.dtype, t.device) for t in batch)

    def _eager(self, batch):
        self.optimizer.zero_grad(set_to_none=True)
        out = self.body(*batch)
        if self.grad_sync is not None:
            self.grad_sync(*batch)
        self.optimizer.step()
        self.eager_steps += 1
        return out

    def _capture(self, batch, key):
        dev = batch[0].device
        self._static = [t.clone() for t in batch]
        self.optimizer.zero_grad(set_to_none=True)   # backward allocates .grad from the graph's pool
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._out = self.body(*self._static)
            if self.grad_sync is None:
                self.optimizer.step()
        self._g_fb = g
        self._grads = [p.grad for p in self.params]
        if self.grad_sync is not None:
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, pool=g.pool()):
                self.optimizer.step()
            self._g_opt = g2
        self._key = key
        torch.cuda.current_stream(dev).synchronize()

    def _replay(self, batch):
        for s, t in zip(self._static, batch):
            s.copy_(t)
        for p, gr in zip(self.params, self._grads):
            p.grad = gr
        self._g_fb.replay()
        if self.grad_sync is not None:
            self.grad_sync(*batch)
            self._g_opt.replay()
        self.replays += 1
        return self._out

    def skip_empty(self, *batch):
        """An EMPTY shard (more ranks than trajectories in a short last batch): no body, but with a ``grad_sync``
        hook the rank still joins the all-reduce (which gives it everyone's gradient) and steps, exactly as
        ``train_model``'s eager loop does — the other ranks' all-reduce would otherwise wait for it forever."""
        if self.grad_sync is None:
            return
        self.optimizer.zero_grad(set_to_none=True)
        self.grad_sync(*batch)
        self.optimizer.step()

    def __call__(self, *batch):
        if not batch or not all(isinstance(t, torch.Tensor) and t.is_cuda for t in batch):
            raise RuntimeError("CapturedStep: the batch must be ROCm device tensors")
        key = self._shape_key(batch)
        if self._g_fb is not None and key == self._key:
            return self._replay(batch)
        if self._g_fb is None and self.eager_steps >= self.warmup:
            self._capture(batch, key)
            return self._replay(batch)
        if self._g_fb is None:
            # warm-up steps on a side stream, as the capture itself runs on one
            dev = batch[0].device
            cur = torch.cuda.current_stream(dev)
            side = torch.cuda.Stream(dev)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                out = self._eager(batch)
            cur.wait_stream(side)
            for t in out:
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(cur)
            return out
        return self._eager(batch)   # another batch shape: the same step, launched eagerly
