"""GPU check of the config-5 gradient product kernel (fcr_wbwd.h) in isolation: random W (4H x NO) and dgates
(B x 4H) split into f16 halves exactly as the rollout splits them; the kernel's fp32 output against the fp64
product of the UNSPLIT fp32 operands (the split's own error is ~2^-22 relative). Also times it.
    python scripts/wb_check.py lib_ab/wbtest.so"""
import ctypes
import sys

import torch

lib = ctypes.CDLL(sys.argv[1])
vp, i32 = ctypes.c_void_p, ctypes.c_int
lib.wb_run.argtypes = [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp]
dev = "cuda"
for (B, H, NO_f, gs) in [(8, 256, 1, 0.3), (8, 256, 2, 0.3), (8, 256, 1, 0.5), (8, 256, 2, 1e-3), (300, 64, 2, 0.3), (1000, 128, 1, 0.3), (65536, 256, 2, 0.3),
                         (65536, 256, 1, 0.3)]:
    torch.manual_seed(0)
    K, NO = 4 * H, NO_f * H
    W = ((torch.rand(K, NO, device=dev) * 2 - 1) / H ** 0.5)
    G = torch.randn(B, K, device=dev) * gs * torch.rand(B, K, device=dev) ** 4   # heavy small-value tail
    Wt = W.t().contiguous()
    whi = Wt.half()
    wlo = (Wt - whi.float()).half()
    ghi = G.half()
    glo = (G - ghi.float()).half()
    rows = torch.empty(B, 12 * H, dtype=torch.half, device=dev)   # the rollout's [hi | lo | -] dgate rows
    rows[:, :K] = ghi
    rows[:, K:2 * K] = glo
    out = torch.full((B, NO + 8), float("nan"), device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    rc = lib.wb_run(p(whi), p(wlo), p(rows), p(out), K, 12 * H, K, NO + 8, B, NO, K, st)
    torch.cuda.synchronize()
    assert rc == 0, rc
    ref = G.double() @ W.double()
    got = out[:, :NO].double()
    err = float((got - ref).abs().max() / ref.abs().max())
    # against the split operands' own three products (the arithmetic the kernel runs, lo x lo dropped)
    gh, gl, wh, wl = ghi.double(), glo.double(), whi.double().t(), wlo.double().t()
    ref3 = gh @ wh + gl @ wh + gh @ wl
    err3 = float((got - ref3).abs().max() / ref3.abs().max())
    untouched = bool(torch.isnan(out[:, NO:]).all())
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(10):
        lib.wb_run(p(whi), p(wlo), p(rows), p(out), K, 12 * H, K, NO + 8, B, NO, K, st)
    ev[1].record()
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) * 100
    tf = 3 * 2.0 * B * NO * K / (us * 1e-6) / 1e12
    print(f"B={B} H={H} NO={NO} gscale={gs}: max rel err {err:.2e} (vs split products {err3:.2e}), padding untouched {untouched}, {us:.1f} us, {tf:.0f} TF/s executed",
          flush=True)

# leftover test: the same call right after a call on DIFFERENT operands (LDS is not cleared between workgroups)
for (B, H, NO_f) in [(8, 256, 1), (8, 256, 2), (4096, 256, 2)]:
    K, NO = 4 * H, NO_f * H
    res = []
    for seed in (1, 2, 1):
        torch.manual_seed(seed)
        W = ((torch.rand(K, NO, device=dev) * 2 - 1) / H ** 0.5)
        G = torch.randn(B, K, device=dev) * 0.3
        Wt = W.t().contiguous()
        whi = Wt.half()
        wlo = (Wt - whi.float()).half()
        rows = torch.empty(B, 12 * H, dtype=torch.half, device=dev)
        rows[:, :K] = G.half()
        rows[:, K:2 * K] = (G - G.half().float()).half()
        out = torch.zeros((B, NO), device=dev)
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        lib.wb_run(p(whi), p(wlo), p(rows), p(out), K, 12 * H, K, NO, B, NO, K,
                   ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        ref = G.double() @ W.double()
        res.append(float((out.double() - ref).abs().max() / ref.abs().max()))
    print(f"leftover test B={B} NO={NO}: errors of seed 1, then seed 2, then seed 1 again: {res}", flush=True)

# bounds test: output rows beyond B and columns beyond NO (ldo = 2H as the rollout's D slabs) must stay untouched
for (B, H, NO) in [(8, 256, 256), (8, 256, 512), (300, 256, 256), (130, 64, 128)]:
    K = 4 * H
    torch.manual_seed(3)
    W = ((torch.rand(K, NO, device=dev) * 2 - 1) / H ** 0.5)
    G = torch.randn(B, K, device=dev) * 0.3
    Wt = W.t().contiguous()
    whi, rows = Wt.half(), torch.empty(B, 12 * H, dtype=torch.half, device=dev)
    wlo = (Wt - whi.float()).half()
    rows[:, :K] = G.half()
    rows[:, K:2 * K] = (G - G.half().float()).half()
    ldo = 2 * H
    out = torch.full((B + 200, ldo), float("nan"), device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    lib.wb_run(p(whi), p(wlo), p(rows), p(out), K, 12 * H, K, ldo, B, NO, K, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    ref = G.double() @ W.double()
    err = float((out[:B, :NO].double() - ref).abs().max() / ref.abs().max())
    rows_ok = bool(torch.isnan(out[B:]).all())
    cols_ok = bool(torch.isnan(out[:B, NO:]).all())
    print(f"bounds B={B} H={H} NO={NO} ldo={ldo}: err {err:.2e}, rows beyond B untouched {rows_ok}, cols beyond NO untouched {cols_ok}",
          flush=True)
