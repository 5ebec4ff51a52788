"""torch.autograd.Function over the gfx950 rollout kernels (C ABI in include/fcr.h).

Forward  = MPCLoss.forward  (/root/reference/Unsupervised Learning/Functions.py:1353-1472)
Backward = what loss.backward() (Functions.py:655) delivers for it: d loss/d u0 (flows on into the
caller's ``controller(X)`` graph) and the gradients of the controller parameters used inside the
loss. The frozen LSTM's weight gradients are not produced (the reference computes them but nothing
consumes them: UL/Main.py:195 optimises the controller only).
"""
from __future__ import annotations

import ctypes

import torch

from . import _native

WINDOW_ROWS = 10   # Functions.py:1434 hard-codes the 10-row window


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def make_dims(B, N, H, layers, ctrl_hidden, alpha, in_dim=5, out_dim=4, ctrl_in=3, L=WINDOW_ROWS, precision=0):
    return _native.FcrDims(B, N, L, H, layers, in_dim, out_dim, ctrl_in, ctrl_hidden, float(alpha), int(precision))


def _dev_f32(t, name):
    if t.dtype != torch.float32:
        raise TypeError(f"{name}: expected float32, got {t.dtype}")
    return t.contiguous()


class CallInfo:
    """What one rollout call ran: its per-call options (fcr_options, carried from the forward to its backward, which
    torch may run on its autograd thread) and the kernel family each pass launched."""

    def __init__(self, opts):
        self.opts = opts
        self.forward = self.backward = None   # "small", "fused" or "wide" once the pass has run
        self.small_batch_limit = None         # the limit both passes ran with (an inherited one resolved by the forward)
        self.workspace_bytes = 0
        self.kept_windows = 0


class RolloutFn(torch.autograd.Function):
    """Inputs: X (B,3), u0 (B,1), states (B,10,5), noise (B,N,4) or None, controller params
    (W_inp, b_inp, W_out), LSTM weights (w_ih0..2, w_hh0..2, fc_w, fc_b), N, alpha, precision, and a CallInfo
    (the call's fcr_options in, the kernel families out).
    Outputs: loss (0-d), cost (B,), command (B,), error (B,), prediction (B*N,), xhat (B,N,4)."""

    @staticmethod
    def forward(ctx, X, u0, states, noise, W_inp, b_inp, W_out, w_ih0, w_ih1, w_ih2, w_hh0, w_hh1,
                w_hh2, fc_w, fc_b, N, alpha, precision=0, info=None):
        lib = _native.load()
        dev = X.device
        B = X.shape[0]
        H = w_hh0.shape[1]
        dims = make_dims(B, N, H, 3, W_inp.shape[0], alpha, precision=precision)
        need_grad = any(ctx.needs_input_grad[i] for i in (1, 4, 5, 6))
        if info is None:
            info = CallInfo(_native.make_options())
        # the small-batch limit resolved ONCE, here: an inherited limit is read from the process-wide default now,
        # and the backward (possibly on the autograd thread, after the caller changed that default) runs with the
        # same value, so both passes pick their kernel family from one limit
        small = info.opts.small_batch_limit
        if small < 0:
            small = int(lib.fcr_get_small_batch_limit())
        opts = _native.FcrOptions(small, 0, info.opts.wide_keep_budget)
        try:
            ws = torch.empty(_native.workspace_bytes(dims, need_grad, opts), dtype=torch.uint8, device=dev)
        except torch.cuda.OutOfMemoryError:
            # H > 52: the kept windows did not fit beside the caller's tensors; the floor workspace recomputes every
            # window instead (the kernels derive the count from ws_bytes). This call's options only.
            floor = _native.FcrOptions(opts.small_batch_limit, 0, 0)
            ws = torch.empty(_native.workspace_bytes(dims, need_grad, floor), dtype=torch.uint8, device=dev)
        info.workspace_bytes = ws.numel()
        info.kept_windows = _native.kept_windows(dims, ws.numel()) if need_grad else 0
        f32 = dict(dtype=torch.float32, device=dev)
        loss = torch.empty((), **f32)
        cost = torch.empty(B, **f32)
        command = torch.empty(B, **f32)
        error = torch.empty(B, **f32)
        prediction = torch.empty(B * N, **f32)
        xhat = torch.empty(B, N, 4, **f32)
        w = _native.FcrWeights()
        keep = [t.contiguous() for t in (W_inp, b_inp, W_out, w_ih0, w_ih1, w_ih2, w_hh0, w_hh1, w_hh2,
                                         fc_w, fc_b)]
        w.ctrl_w_inp, w.ctrl_b_inp, w.ctrl_w_out = (t.data_ptr() for t in keep[0:3])
        for l in range(3):
            w.w_ih[l] = keep[3 + l].data_ptr()
            w.w_hh[l] = keep[6 + l].data_ptr()
        w.fc_w, w.fc_b = keep[9].data_ptr(), keep[10].data_ptr()
        Xc, u0c, stc = X.contiguous(), u0.contiguous(), states.contiguous()
        nzc = noise.contiguous() if noise is not None else None
        _native.check(lib.fcr_forward(ctypes.byref(dims), ctypes.byref(opts), ctypes.byref(w), _ptr(Xc), _ptr(u0c),
                                      _ptr(stc), _ptr(nzc), _ptr(loss), _ptr(cost), _ptr(command), _ptr(error),
                                      _ptr(prediction), _ptr(xhat), int(need_grad), _ptr(ws), ws.numel(),
                                      _stream(dev)), "fcr_forward")
        info.forward, info.backward = _native.KERNEL_FAMILIES[opts.kernels], None
        info.small_batch_limit = small
        ctx.mark_non_differentiable(cost, command, error, prediction, xhat)
        # only loss carries a gradient: without this autograd launches a zero-fill kernel per output
        # before every backward (six per step, ~3 us each at the reference's B = 15)
        ctx.set_materialize_grads(False)
        if need_grad:
            ctx.ws = ws
            ctx.dims = dims
            ctx.info = info
            ctx.small_limit = small
            ctx.save_for_backward(Xc, stc, prediction)
            ctx.ctrl_shapes = (W_inp.shape, b_inp.shape, W_out.shape)
        return loss, cost, command, error, prediction, xhat

    @staticmethod
    def backward(ctx, g_loss, *unused):
        if g_loss is None:   # (materialize_grads off) nothing flowed into loss
            ctx.ws = None
            return (None,) * 19
        if ctx.ws is None:
            raise RuntimeError("MPCLoss: trying to backward through the same rollout a second time; its workspace (the "
                               "saved sequence slabs) was released by the first backward: recompute the loss")
        lib = _native.load()
        Xc, stc, prediction = ctx.saved_tensors
        dev = Xc.device
        B = Xc.shape[0]
        f32 = dict(dtype=torch.float32, device=dev)
        g_u0 = torch.empty(B, 1, **f32)
        s_wi, s_bi, s_wo = ctx.ctrl_shapes
        g_wi = torch.empty(s_wi, **f32)
        g_bi = torch.empty(s_bi, **f32)
        g_wo = torch.empty(s_wo, **f32)
        dl = g_loss.detach().to(torch.float32).reshape(1).contiguous()
        info = ctx.info
        # the call's options; an inherited small-batch limit is the value the forward resolved (no process state is
        # read here, so a default changed in between on another thread does not split the passes)
        small = info.opts.small_batch_limit if info.opts.small_batch_limit >= 0 else ctx.small_limit
        opts = _native.FcrOptions(small, 0, info.opts.wide_keep_budget)
        _native.check(lib.fcr_backward(ctypes.byref(ctx.dims), ctypes.byref(opts), _ptr(Xc), _ptr(stc),
                                       _ptr(prediction), _ptr(dl), _ptr(g_u0), _ptr(g_wi), _ptr(g_bi), _ptr(g_wo),
                                       _ptr(ctx.ws), ctx.ws.numel(), _stream(dev)), "fcr_backward")
        info.backward = _native.KERNEL_FAMILIES[opts.kernels]
        ctx.ws = None   # release the activation slab as early as autograd lets us
        return (None, g_u0, None, None, g_wi, g_bi, g_wo) + (None,) * 12


PRECISIONS = {"fp32": _native.PRECISION_FP32, "f16": _native.PRECISION_F16}


def rollout(X, u0, states, ctrl_params, lstm_params, N, alpha, noise=None, precision="fp32", info=None):
    """Functional entry: ctrl_params = (W_inp, b_inp, W_out), lstm_params = (w_ih[3], w_hh[3], fc_w, fc_b).
    precision: "fp32" (fp32-accurate, the default) or "f16" (config 3: f16 gate products in both passes, fp32
    accumulate, include/fcr.h FCR_PRECISION_F16; the former "f16fwd" mode is retired). info: a CallInfo with this call's fcr_options (None: every option inherits the process
    default); the kernel families it ran are recorded in it."""
    if precision not in PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {precision!r}")
    w_ih, w_hh, fc_w, fc_b = lstm_params
    dev = X.device
    if dev.type != "cuda":
        raise RuntimeError("forging-control_amd rollout runs on a ROCm device only (got %s); the CPU "
                           "restatement in oracle/ is test infrastructure, not a fallback" % dev)
    tensors = [X, u0, states] + list(ctrl_params) + list(w_ih) + list(w_hh) + [fc_w, fc_b]
    for t in tensors:
        if t.device != dev:
            raise RuntimeError(f"all rollout tensors must be on {dev}, found one on {t.device}")
    if states.dim() != 3 or states.shape[1] != WINDOW_ROWS or states.shape[2] != 5:
        raise ValueError(f"states must be (B, 10, 5), got {tuple(states.shape)}")
    B = X.shape[0]
    if X.shape != (B, 3) or u0.numel() != B:
        raise ValueError(f"X must be (B,3) and u0 (B,1); got {tuple(X.shape)}, {tuple(u0.shape)}")
    if noise is not None and noise.shape != (B, N, 4):
        raise ValueError(f"noise must be (B, N, 4) = {(B, N, 4)}, got {tuple(noise.shape)}")
    u0 = u0.reshape(B, 1)
    return RolloutFn.apply(_dev_f32(X, "X"), _dev_f32(u0, "u0"), _dev_f32(states, "states"),
                           None if noise is None else _dev_f32(noise, "noise"),
                           *[_dev_f32(t, "controller param") for t in ctrl_params],
                           *[_dev_f32(t, "lstm weight") for t in list(w_ih) + list(w_hh) + [fc_w, fc_b]],
                           int(N), float(alpha), PRECISIONS[precision], info)
