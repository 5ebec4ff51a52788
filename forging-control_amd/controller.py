"""The caller's controller call on gfx950: ``output = model(X)`` (/root/reference/Unsupervised Learning/
Functions.py:643), i.e. FNNModel.forward (Functions.py:261-289) at the reference's shape —
Linear(3 -> hidden) + ReLU, Linear(hidden -> 1, no bias), Hardtanh (UL/Main.py:188, width_dim = 1) —
and its autograd backward, through fcr_fnn_forward / fcr_fnn_backward (include/fcr.h).

Torch ran this call as rocBLAS GEMMs (~0.33 ms of a 9.5 ms B = 65 536 training step, most of it the
backward's batch reductions); the HIP kernels take microseconds. Other FNNModel shapes (width > 1,
other activations, no bias) are not the hot path and run as the module's own torch layers.
"""
from __future__ import annotations

import ctypes

import torch
from torch import nn

from . import _native

MAX_HIDDEN = 64   # fcr_fnn.h kFnnMaxHidden


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class FNNFunction(torch.autograd.Function):
    """u = Hardtanh(W_out · ReLU(W_inp · x + b_inp)) for X (B,3) -> (B,1)."""

    @staticmethod
    def forward(ctx, X, W_inp, b_inp, W_out):
        lib = _native.load()
        Xc, Wi, bi, Wo = (t.contiguous() for t in (X, W_inp, b_inp, W_out))
        B, hidden = Xc.shape[0], Wi.shape[0]
        u = torch.empty(B, 1, dtype=torch.float32, device=Xc.device)
        _native.check(lib.fcr_fnn_forward(B, Xc.shape[1], hidden, _ptr(Xc), _ptr(Wi), _ptr(bi), _ptr(Wo), _ptr(u),
                                          _stream(Xc.device)), "fcr_fnn_forward")
        ctx.save_for_backward(Xc, Wi, bi, Wo)
        return u

    @staticmethod
    def backward(ctx, g_u):
        lib = _native.load()
        Xc, Wi, bi, Wo = ctx.saved_tensors
        B, hidden = Xc.shape[0], Wi.shape[0]
        dev = Xc.device
        f32 = dict(dtype=torch.float32, device=dev)
        g_X = torch.empty(B, Xc.shape[1], **f32) if ctx.needs_input_grad[0] else None
        g_Wi, g_bi, g_Wo = torch.empty_like(Wi), torch.empty_like(bi), torch.empty_like(Wo)
        nbytes = ctypes.c_size_t(0)
        _native.check(lib.fcr_fnn_workspace_size(B, hidden, ctypes.byref(nbytes)), "fcr_fnn_workspace_size")
        ws = torch.empty(max(int(nbytes.value), 4), dtype=torch.uint8, device=dev)
        gu = g_u.detach().to(torch.float32).contiguous()
        _native.check(lib.fcr_fnn_backward(B, Xc.shape[1], hidden, _ptr(Xc), _ptr(Wi), _ptr(bi), _ptr(Wo), _ptr(gu),
                                           _ptr(g_X), _ptr(g_Wi), _ptr(g_bi), _ptr(g_Wo), _ptr(ws), ws.numel(),
                                           _stream(dev)), "fcr_fnn_backward")
        return g_X, g_Wi, g_bi, g_Wo


def hip_shape_ok(model, x) -> bool:
    """True when ``model(x)`` is the reference's controller shape on a ROCm device (the HIP path)."""
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.shape[1] == 3
            and model.width_dim == 1 and isinstance(model.activation, nn.ReLU)
            and model.fc_inp.bias is not None and model.fc_out.out_features == 1
            and 1 <= model.fc_inp.out_features <= MAX_HIDDEN
            and all(p.dtype == torch.float32 and p.device == x.device
                    for p in (model.fc_inp.weight, model.fc_inp.bias, model.fc_out.weight)))


def fnn_apply(model, x):
    return FNNFunction.apply(x, model.fc_inp.weight, model.fc_inp.bias, model.fc_out.weight)
