"""GPU: the caller's controller call `model(X)` (Functions.py:643; FNNModel.forward :261-289) on the HIP
kernels (fcr_fnn_forward / fcr_fnn_backward) against fp64 torch autograd of the same module."""
import numpy as np
import pytest
import torch

import forging_control_amd as fca
from conftest import relerr

pytestmark = pytest.mark.gpu


def reference(X, Wi, bi, Wo, g):
    """fp64 torch autograd of Hardtanh(W_out ReLU(W_inp x + b)) — the reference module's arithmetic."""
    t = [torch.tensor(a, dtype=torch.float64, requires_grad=True) for a in (X, Wi, bi, Wo)]
    u = torch.nn.functional.hardtanh(torch.relu(t[0] @ t[1].T + t[2]) @ t[3].T)
    u.backward(torch.tensor(g, dtype=torch.float64))
    return u.detach().numpy(), [x.grad.numpy() for x in t]


@pytest.mark.parametrize("B,hidden,scale,x_grad", [
    (1, 50, 1.0, False), (15, 50, 1.0, True), (257, 1, 1.0, False), (4099, 64, 1.0, True),
    (65536, 50, 1.0, False), (3000, 50, 6.0, True),   # scale 6: most outputs clip at +-1 (Hardtanh' = 0)
])
def test_fnn_matches_fp64_autograd(B, hidden, scale, x_grad):
    dev = torch.device("cuda", 0)
    gen = np.random.default_rng(B * 131 + hidden)
    X = gen.uniform(-1, 1, (B, 3)).astype(np.float32)
    torch.manual_seed(B * 131 + hidden)   # the module's Xavier init: fixed, so the sums' conditioning is too
    m = fca.FNNModel(3, hidden, 1, 1).to(dev)
    with torch.no_grad():
        m.fc_inp.weight.mul_(scale)
        m.fc_inp.bias.copy_(torch.tensor(gen.uniform(-0.3, 0.3, hidden), dtype=torch.float32))
        m.fc_out.weight.mul_(scale)
    Xd = torch.tensor(X, device=dev, requires_grad=x_grad)
    g = gen.standard_normal((B, 1)).astype(np.float32)
    u = m(Xd)
    assert u.grad_fn is not None and type(u.grad_fn).__name__.startswith("FNNFunction")
    u.backward(torch.tensor(g, device=dev))
    Wi, bi, Wo = (p.detach().cpu().numpy() for p in (m.fc_inp.weight, m.fc_inp.bias, m.fc_out.weight))
    u_ref, (gX, gWi, gbi, gWo) = reference(X, Wi, bi, Wo, g)
    assert relerr(u.detach().cpu().numpy(), u_ref) <= 1e-5   # fp32 sums of 50 products
    assert relerr(m.fc_inp.weight.grad.cpu().numpy(), gWi) <= 1e-5
    assert relerr(m.fc_inp.bias.grad.cpu().numpy(), gbi) <= 1e-5
    assert relerr(m.fc_out.weight.grad.cpu().numpy(), gWo) <= 1e-5
    if x_grad:
        assert relerr(Xd.grad.cpu().numpy(), gX) <= 1e-5
    if scale > 1:
        assert (np.abs(u_ref) >= 1).mean() > 0.3   # the clipped branch is exercised


def test_fnn_deterministic_and_empty_batch():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = fca.FNNModel(3, 50, 1, 1).to(dev)
    X = torch.rand(10000, 3, device=dev) * 2 - 1
    grads = []
    for _ in range(2):
        m.zero_grad()
        m(X).sum().backward()
        grads.append(torch.cat([p.grad.flatten() for p in (m.fc_inp.weight, m.fc_inp.bias, m.fc_out.weight)]))
    assert torch.equal(grads[0], grads[1])
    m.zero_grad()
    u = m(torch.empty(0, 3, device=dev))
    u.sum().backward()
    assert u.shape == (0, 1) and float(m.fc_inp.weight.grad.abs().sum()) == 0.0
