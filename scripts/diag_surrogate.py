"""Per-tensor relative errors of the surrogate step at H=256 (diagnostic)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
from test_surrogate import params_for, batch, model_for, grads_of
from oracle import surrogate_torch as S
from conftest import relerr
for H, B in ((256, 64), (256, 1024), (128, 64), (50, 64)):
    p = params_for(H, seed=H); x, t = batch(B, seed=B + H)
    _, _, gr = S.step_grads(p, x, t)
    m = model_for(p)
    y = m(torch.tensor(x, dtype=torch.float32, device="cuda:0"), "cuda:0")
    torch.nn.functional.mse_loss(y, torch.tensor(t, dtype=torch.float32, device="cuda:0")).backward()
    g = grads_of(m)
    # torch's own fp32 GPU path for comparison
    tm = S.build(p, torch.float32).to("cuda:0")
    yt = tm(torch.tensor(x, dtype=torch.float32, device="cuda:0"))
    torch.nn.functional.mse_loss(yt, torch.tensor(t, dtype=torch.float32, device="cuda:0")).backward()
    print(H, B, "ours Wih", [f"{relerr(g['Wih'][k], gr['Wih'][k]):.2e}" for k in range(3)],
          "Whh", [f"{relerr(g['Whh'][k], gr['Whh'][k]):.2e}" for k in range(3)])
    print(H, B, "torch-gpu Wih", [f"{relerr(getattr(tm.lstm, f'weight_ih_l{k}').grad.cpu().numpy(), gr['Wih'][k]):.2e}" for k in range(3)],
          "Whh", [f"{relerr(getattr(tm.lstm, f'weight_hh_l{k}').grad.cpu().numpy(), gr['Whh'][k]):.2e}" for k in range(3)])
