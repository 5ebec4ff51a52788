"""LSTM surrogate training on the gfx950 path.

The reference trains the plant surrogate ``LSTMModel(5, 50, 4, 3)`` with ``nn.MSELoss`` and AdamW
(Model_NN/Main.py:218-242) through ``NeuralNetwork.train_model`` (Model_NN/Functions.py:520-569), i.e.
``output = model(X, device); loss = loss_function(output, y.squeeze()); loss.backward();
optimizer.step()`` per batch. Here ``LSTMModel.forward`` on a ROCm device runs :class:`LSTMFunction`:
``fcr_lstm_forward`` and, on ``backward``, ``fcr_lstm_backward``. For H <= 52 (the reference's H = 50)
they are the rollout's fused split-f16 cell kernels over one window (csrc/fcr_sur.h: one forward launch,
one backward launch that also keeps every cell's dgates, and one hand-written weight-gradient product per
layer over all 10·B (step, sample) rows); wider models run the per-cell path (csrc/fcr_wide.h). Every
LSTM weight, the readout and — when it requires grad — the input window receive gradients, so the
reference's loop and optimizer run unchanged.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native
from .rollout import WINDOW_ROWS, make_dims


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _weights(w_ih, w_hh, fc_w, fc_b):
    w = _native.FcrWeights()
    w.w_ih = (ctypes.c_void_p * 3)(*[t.data_ptr() for t in w_ih])
    w.w_hh = (ctypes.c_void_p * 3)(*[t.data_ptr() for t in w_hh])
    w.fc_w, w.fc_b = fc_w.data_ptr(), fc_b.data_ptr()
    return w


class LSTMFunction(torch.autograd.Function):
    """y = LSTMModel(x) with gradients for x and every weight (fcr_lstm_forward / fcr_lstm_backward)."""

    @staticmethod
    def forward(ctx, x, w_ih0, w_ih1, w_ih2, w_hh0, w_hh1, w_hh2, fc_w, fc_b):
        dev = x.device
        B, H = x.shape[0], w_hh0.shape[1]
        dims = make_dims(B, 1, H, 3, 1, 0.0)
        ts = [t.detach().to(torch.float32).contiguous() for t in (x, w_ih0, w_ih1, w_ih2, w_hh0, w_hh1, w_hh2, fc_w, fc_b)]
        xc, w_ih, w_hh, fcw, fcb = ts[0], ts[1:4], ts[4:7], ts[7], ts[8]
        w = _weights(w_ih, w_hh, fcw, fcb)
        need_grad = any(ctx.needs_input_grad)
        lib = _native.load()
        nbytes = ctypes.c_size_t(0)
        _native.check(lib.fcr_lstm_workspace_size(ctypes.byref(dims), int(need_grad), ctypes.byref(nbytes)),
                      "fcr_lstm_workspace_size")
        ws = torch.empty(nbytes.value, dtype=torch.uint8, device=dev)
        y = torch.empty(B, 4, dtype=torch.float32, device=dev)
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _native.check(lib.fcr_lstm_forward(ctypes.byref(dims), ctypes.byref(w), _p(xc), _p(y), int(need_grad),
                                           _p(ws), ws.numel(), stream), "fcr_lstm_forward")
        if need_grad:
            ctx.dims, ctx.ws, ctx.tensors = dims, ws, ts
        return y

    @staticmethod
    def backward(ctx, dy):
        ts = ctx.tensors
        xc, w_ih, w_hh, fcw, fcb = ts[0], ts[1:4], ts[4:7], ts[7], ts[8]
        dev = xc.device
        g = [torch.empty_like(t) for t in ts]
        w = _weights(w_ih, w_hh, fcw, fcb)
        g_ih = (ctypes.c_void_p * 3)(*[t.data_ptr() for t in g[1:4]])
        g_hh = (ctypes.c_void_p * 3)(*[t.data_ptr() for t in g[4:7]])
        dyc = dy.to(torch.float32).contiguous()
        lib = _native.load()
        _native.check(lib.fcr_lstm_backward(ctypes.byref(ctx.dims), ctypes.byref(w), _p(dyc), g_ih, g_hh, _p(g[7]),
                                            _p(g[8]), _p(g[0]) if ctx.needs_input_grad[0] else None, _p(ctx.ws),
                                            ctx.ws.numel(), ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
                      "fcr_lstm_backward")
        return tuple(gi if need else None for gi, need in zip(g, ctx.needs_input_grad))


def hip_shape_ok(model, x) -> bool:
    """True when ``model(x)`` is the shape the gfx950 LSTM path is built for: LSTM(5, H, 3) without LSTM
    bias -> Linear(H, 4), fp32 (B, 10, 5) windows on the device the weights live on."""
    lstm = model.lstm
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3 and tuple(x.shape[1:]) == (WINDOW_ROWS, 5)
            and not lstm.bias and lstm.num_layers == 3 and lstm.input_size == 5 and model.fc.out_features == 4
            and lstm.batch_first and all(p.dtype == torch.float32 and p.device == x.device for p in model.parameters()))


def lstm_apply(model, x: torch.Tensor) -> torch.Tensor:
    """LSTMModel forward on the HIP path (x (B, 10, 5) on a ROCm device); :func:`hip_shape_ok` must hold."""
    if not hip_shape_ok(model, x):
        raise RuntimeError("the gfx950 LSTM path is built for LSTMModel(5, H, 4, 3) without LSTM bias on fp32 "
                           f"(B, 10, 5) device windows (Model_NN/Main.py:225, UL/Main.py:144-154); got {tuple(x.shape)} "
                           f"on {x.device}")
    lstm = model.lstm
    p = [getattr(lstm, f"weight_ih_l{k}") for k in range(3)] + [getattr(lstm, f"weight_hh_l{k}") for k in range(3)]
    return LSTMFunction.apply(x, *p, model.fc.weight, model.fc.bias)


def captured_step(model, loss_function, optimizer, device, warmup=2):
    """The batch step of :func:`train_model` as a :class:`~.graphed.CapturedStep` (one HIP graph replay
    per batch; pass it as ``train_model(..., step=...)``)."""
    from .graphed import CapturedStep

    def body(X, y):
        loss = loss_function(model(X, device), y.squeeze())
        loss.backward()
        return (loss.detach(),)

    return CapturedStep(model.parameters(), optimizer, body, None, warmup)


def train_model(data_loader, model, loss_function, optimizer, device, step=None):
    """Model_NN/Functions.py:520-569 with the same arguments and return value (average batch loss).
    ``step`` (optional, from :func:`captured_step`) replays each batch from a HIP graph and reads the
    summed loss once per epoch instead of once per batch."""
    model.train()
    if step is not None:
        total_dev = None
        for X, y in data_loader:
            (loss,) = step(X.to(device), y.to(device))
            total_dev = loss.clone() if total_dev is None else total_dev + loss
        return (float(total_dev.item()) if total_dev is not None else 0.0) / len(data_loader)
    total = 0.0
    for X, y in data_loader:
        X, y = X.to(device), y.to(device)
        optimizer.zero_grad()
        output = model(X, device)
        loss = loss_function(output, y.squeeze())
        loss.backward()
        optimizer.step()
        total += loss.item()
    return total / len(data_loader)
