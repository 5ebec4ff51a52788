"""Benchmark: one optimizer step of the unsupervised-MPC training path on the gfx950 rollout engine.

A step = controller(X) -> MPCLoss rollout (fused HIP forward) -> loss.backward() (fused HIP backward)
-> RCCL all-reduce of the controller gradients (N > 1 GPUs) -> AdamW, exactly the body of
NeuralNetwork.train_model (/root/reference/Unsupervised Learning/Functions.py:640-661).

Workload (BASELINE.json configs[1]): B = 65 536 trajectories per GPU, horizon N = 10, LSTM hidden 50
(3 layers, the reference's trained surrogate weights from tests/golden/weights_ref.npz), controller
3->50->1, fp32. Weak scaling: every rank runs its own 65 536 trajectories.

Prints ONE JSON line (rank 0). See DESIGN.md §Measurement for the roofline definitions.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import forging_control_amd as fca  # noqa: E402

FP32_PEAK_TFLOPS = 157.3          # MI355X dense FP32 (vector = MFMA), MI355X_MICROARCH.md
F16_PEAK_TFLOPS = 2500.0          # MI355X dense FP16/BF16 MFMA (no sparsity), MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0             # MI355X HBM3E spec
ALPHA = 20.0                      # UL/Main.py:192
GRAD_CHECK_BUDGET_S = 300.0       # rank 0's post-timing check of its shard; the process group waits 30 min


def flops_per_rollout_step(H=50, L=10, layers=3, in_dim=5, ctrl_hidden=50):
    """Algorithmic FLOP of one (trajectory, horizon step): SURVEY.md §8(a3)/(d).
    Forward LSTM call: 2*[L*4H*(in+H) + (layers-1)*L*8H^2 + 4H] (readout incl.); controller 2*(3*50+50);
    backward input-gradient products: the same LSTM contraction count again (W^T . dgates)."""
    lstm = 2 * (L * 4 * H * (in_dim + H) + (layers - 1) * L * 8 * H * H + 4 * H)
    fnn = 2 * (3 * ctrl_hidden + ctrl_hidden)
    return {"fwd": lstm + fnn, "bwd": lstm + fnn, "total": 2 * (lstm + fnn)}


def hbm_bytes_per_rollout_step(N=10):
    """Compulsory HBM bytes per rollout-step: X 12 + states 200 + outputs 12 + 4N per
    trajectory, divided by N."""
    return (12 + 200 + 3 * 4 + 4 * N) / N


def pmc_traffic(kernel, suffix=""):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary of this workload
    (profiles/round<k><suffix>_pmc.json, scripts/profile_round.sh; older profiles/r<k>_pmc.json otherwise), or
    None. suffix "_c3f16" / "_c3fp32": config 3's summaries (scripts/profile.sh c3 / c3f16); "_c5": config 5's summary, whose "bwd_pass" entry is the HBM bytes of one whole backward pass."""
    import glob
    import re
    pick = []
    for f in glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")):
        m = re.fullmatch(r"(round|r)(\d+)([a-z]?)" + suffix + r"_pmc\.json", os.path.basename(f))   # the rollout's
        if m:
            pick.append((m.group(1) == "round", int(m.group(2)), m.group(3), f))
    if not pick:
        return None, None
    f = max(pick)[-1]
    d = json.load(open(f))
    if kernel not in d or not d[kernel].get("hbm_bytes_corrected"):
        return None, None
    return d[kernel]["hbm_bytes_corrected"], os.path.basename(f)


WEIGHT_KEYS = ("Wih0", "Wih1", "Wih2", "Whh0", "Whh1", "Whh2", "fcW", "fcb", "W_inp", "b_inp", "W_out")


def weight_arrays(H):
    """The benchmark's weights as float32 arrays: the reference-trained set at H = 50 (tests/golden), seeded synthetic
    uniform(-1/sqrt(H), 1/sqrt(H)) otherwise."""
    if H == 50:
        w = np.load(os.path.join(ROOT, "tests", "golden", "weights_ref.npz"))
        return {k: np.asarray(w[k], np.float32) for k in WEIGHT_KEYS}
    gen = torch.Generator().manual_seed(0)
    shapes = {"Wih0": (4 * H, 5), "Wih1": (4 * H, H), "Wih2": (4 * H, H), "Whh0": (4 * H, H), "Whh1": (4 * H, H),
              "Whh2": (4 * H, H), "fcW": (4, H), "fcb": (4,), "W_inp": (50, 3), "b_inp": (50,), "W_out": (1, 50)}
    return {k: ((torch.rand(s, generator=gen) * 2 - 1) / np.sqrt(H)).numpy() for k, s in shapes.items()}


def load_weights(dev, H):
    w = weight_arrays(H)
    g = lambda k: torch.as_tensor(w[k])
    sim = fca.LSTMModel(5, H, 4, 3).to(dev)
    ctrl = fca.FNNModel(3, 50, 1, 1).to(dev)
    with torch.no_grad():
        for k in range(3):
            getattr(sim.lstm, f"weight_ih_l{k}").copy_(g(f"Wih{k}"))
            getattr(sim.lstm, f"weight_hh_l{k}").copy_(g(f"Whh{k}"))
        sim.fc.weight.copy_(g("fcW"))
        sim.fc.bias.copy_(g("fcb"))
        ctrl.fc_inp.weight.copy_(g("W_inp"))
        ctrl.fc_inp.bias.copy_(g("b_inp"))
        ctrl.fc_out.weight.copy_(g("W_out"))
    return sim, ctrl


def synth_batch(B, dev, seed):
    """SURVEY.md §8(d) input distribution (synthetic: the reference's Data/ pickle is not shipped)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    X = torch.empty(B, 3)
    X[:, 0].uniform_(-1, 1, generator=g)
    X[:, 1].uniform_(-1, 1, generator=g)
    sign = torch.randint(0, 2, (B,), generator=g).float() * 2 - 1
    X[:, 2] = sign * torch.empty(B).uniform_(0.11, 0.99, generator=g)
    S = torch.empty(B, 10, 5).uniform_(-1, 1, generator=g)
    S[:, :, 1:3].uniform_(0.0, 1.1, generator=g)
    return X.to(dev), S.to(dev)


def host_cpu_info():
    """What the host offers this process: nproc (the machine), the CPUs it may run on (affinity), the
    cgroup CPU quota (the box's share), and lscpu's model name."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = info["nproc"]
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    info["cgroup_cpus"] = quota
    model = None
    try:
        import subprocess
        for line in subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout.splitlines():
            if line.startswith("Model name"):
                model = line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    info["model"] = model
    usable = info["affinity"]
    if quota:
        usable = min(usable, max(1, int(quota)))
    info["usable"] = usable
    return info


def cpu_baseline(budget_s=24.0, N=10, H=50):
    """The reference CPU path (stock torch ops in MPCLoss's order, oracle/rollout_torch.py, with the
    reference's requires_grad on the frozen LSTM) timed on the host: forward + backward + AdamW per step,
    at B = 15 (the reference's training batch, UL/Main.py:84), B = 256 (BASELINE config 1 as written) and
    B = 4 096 (stands in for config 2's B = 65 536: rollout-steps/s is per (trajectory, step), and the CPU
    path is throughput-bound from a few thousand trajectories on), each on all usable host cores and on
    one thread. The reported value is B = 256 at the faster of the two thread counts (torch's intra-op
    threads do not pay at these small per-op sizes on a shared host). At H > 52 (config 5) the same path on the
    line's own N, H and weights, at B = 15 and B = 256 (a B = 256 step is ~1 s of host work there): B = 256 on all
    usable cores only."""
    from oracle import rollout_torch as T
    info = host_cpu_info()
    w = weight_arrays(H)
    params = {"Wih": [w[f"Wih{k}"] for k in range(3)], "Whh": [w[f"Whh{k}"] for k in range(3)], "fcW": w["fcW"],
              "fcb": w["fcb"], "W_inp": w["W_inp"], "b_inp": w["b_inp"], "W_out": w["W_out"]}
    sim, ctrl = T.build_modules(params, torch.float32)
    opt = torch.optim.AdamW(ctrl.parameters(), lr=1e-4)
    runs = []
    wide = H > 52
    share = {15: 0.3, 256: 0.7} if wide else {15: 0.15, 256: 0.35, 4096: 0.5}
    for B in share:
        X, S = synth_batch(B, "cpu", 99)

        def step():
            opt.zero_grad()
            u0 = ctrl(X)
            loss, _ = T.mpc_loss(sim, ctrl, X, u0, S, N, ALPHA)
            loss.backward()
            opt.step()

        for threads in ((info["usable"],) if wide and B > 15 else (info["usable"], 1)):
            torch.set_num_threads(threads)
            step()
            t0 = time.perf_counter()
            iters = 0
            while iters < 1 or (time.perf_counter() - t0 < budget_s * share[B] / 2 and iters < 500):
                step()
                iters += 1
            dt = time.perf_counter() - t0
            runs.append({"batch": B, "threads": threads, "steps": iters, "seconds": round(dt, 3),
                         "rollout_steps_per_s": B * N * iters / dt})
    main_run = max((r for r in runs if r["batch"] == 256), key=lambda r: r["rollout_steps_per_s"])
    return {"value": main_run["rollout_steps_per_s"], "unit": "rollout-steps/s", "cores": main_run["threads"],
            "kind": "port",
            "sample": (f"oracle/rollout_torch.py fwd+bwd+AdamW (reference op order, LSTM weight grads on), N={N} "
                       f"H={H}; value = B=256 at the faster of {info['usable']} threads and 1 thread; B=4096 stands in "
                       f"for B=65536 (per rollout-step rate); torch {torch.__version__}") if not wide else
                      (f"oracle/rollout_torch.py fwd+bwd+AdamW (reference op order, LSTM weight grads on), N={N} "
                       f"H={H}, the line's seeded weights; value = B=256 on {info['usable']} threads (B=15 also on "
                       f"1 thread); per rollout-step rate; torch {torch.__version__}"),
            "runs": runs, "host": info}


# v_mfma_f32_16x16x32_f16 issued per 16-trajectory wave and LSTM cell (layer 0, layers >= 1) in the fp32-accurate
# H <= 52 kernels at HS = 13 (DESIGN.md §2 "Packed tail block"; cross-checked against SQ_INSTS_VALU_MFMA_F16 in
# profiles/round2_pmc.json): the forward's three split products, the backward's recompute + transposed products
MFMA_PER_WAVE_CELL = {"fwd": (78, 130), "bwd": (158, 270)}
MFMA_FLOP = 16 * 16 * 32 * 2


def executed_mfma_flop(kind, B, N, L=10):
    """f16 MFMA FLOP one launch of the fp32-accurate H = 50 kernel executes (padding and recompute included)."""
    waves = (B + 15) // 16
    l0, l12 = MFMA_PER_WAVE_CELL[kind]
    return waves * N * L * (l0 + 2 * l12) * MFMA_FLOP


def grad_check(sim, ctrl, X, S, N, dev, precision, B_check=None):
    """grad fp32 max-rel-err vs the PyTorch restatement (BASELINE.json's metric): the HIP MPCLoss forward +
    backward on the benchmarked batch (u0 = controller(X) as a leaf, as the parity tests take it) against
    oracle/rollout_torch.py in fp64 on the same device, chunked over trajectories. Per tensor
    max|g - g_ref| / max|g_ref|; run after the timed region, as the checker only."""
    from oracle import rollout_torch as T
    if B_check is not None and B_check < X.shape[0]:
        X, S = X[:B_check].contiguous(), S[:B_check].contiguous()
    B = X.shape[0]
    with torch.no_grad():
        u0 = ctrl(X)
    u = u0.detach().clone().requires_grad_(True)
    fn = fca.MPCLoss(prediction_horizon=N, alpha=ALPHA, precision=precision)
    for p in ctrl.parameters():
        p.grad = None
    loss, f = fn(sim, ctrl, X, u, S, dev)
    loss.backward()
    got = {"loss": f["loss"], "prediction": f["prediction"], "xhat": fn.last_trajectory, "g_u0": u.grad.reshape(-1),
           "g_W_inp": ctrl.fc_inp.weight.grad, "g_b_inp": ctrl.fc_inp.bias.grad, "g_W_out": ctrl.fc_out.weight.grad}
    cpu = lambda t: t.detach().double().cpu().numpy()
    params = {"Wih": [cpu(getattr(sim.lstm, f"weight_ih_l{k}")) for k in range(3)],
              "Whh": [cpu(getattr(sim.lstm, f"weight_hh_l{k}")) for k in range(3)],
              "fcW": cpu(sim.fc.weight), "fcb": cpu(sim.fc.bias), "W_inp": cpu(ctrl.fc_inp.weight),
              "b_inp": cpu(ctrl.fc_inp.bias), "W_out": cpu(ctrl.fc_out.weight)}
    H = params["Whh"][0].shape[1]
    ref = T.loss_and_grads_chunked(params, X, u.detach(), S, N, ALPHA, device=dev,
                                   chunk=16384 if H <= 64 else 2048)
    # every output over ALL trajectories (continuous across the ReLU/Hardtanh/constraint kinks) and the full-batch
    # parameter gradients (flips included); per-trajectory g_u0 outside the kink band (trajectories whose fp64
    # rollout passes within 1e-5 of a kink, where an fp32 mask may flip one term's slope: tests/test_gpu_fullsize.py),
    # the band reported on its own beside stock torch fp32's error there
    # the reference's own arithmetic (stock torch fp32, same oracle, same device) against the same fp64: the fp32
    # noise floor of this batch, beside which the HIP errors are to be read
    ref32 = T.loss_and_grads_chunked(params, X, u.detach(), S, N, ALPHA, device=dev, dtype=torch.float32,
                                     chunk=16384 if H <= 64 else 2048)
    reg = T.kink_margin(params, X.double(), ref["xhat"].reshape(B, N, 4)) > 1e-5
    got["prediction"] = got["prediction"].reshape(B, N)
    err = {}
    band = {}
    for k, v in got.items():
        r = ref[k].reshape(v.shape)
        a = v.double()
        den = r.abs().max().clamp_min(1e-300)
        if k == "g_u0":
            e = (a - r).abs() / den
            e32 = (ref32[k].reshape(v.shape).double() - r).abs() / den
            hip_b = float(e[~reg].max()) if (~reg).any() else 0.0
            t32_b = float(e32[~reg].max()) if (~reg).any() else 0.0
            # a band g_u0 above 1e-5 must be the fp64 one-sided derivative of its kink (u0 shifted by +-d): a flip
            flagged = torch.nonzero(~reg & (e > 1e-5)).reshape(-1).tolist()
            # one fp64 rollout per shift and trajectory: the fp32-accurate mode's few flips only
            examine = precision == "fp32" and len(flagged) <= 64
            side = T.one_sided_g_u0(params, X, u.detach(), S, N, ALPHA, flagged, B, device=dev) if examine else {}
            flips = []
            for i in (flagged if examine else []):
                g = float(a[i])
                best = min(side[i], key=lambda sg: abs(g - sg[1]))
                flips.append({"trajectory": i, "err_at_u0": float(e[i]), "one_sided_shift": best[0],
                              "err_one_sided": abs(g - best[1]) / float(den)})
            band = {"trajectories": int((~reg).sum()), "max_rel_err": hip_b, "above_1e-5": len(flagged),
                    "torch_fp32_max_rel_err": t32_b, "torch_fp32_above_1e-5": int((e32[~reg] > 1e-5).sum()),
                    "flips": flips, "flips_examined": examine,
                    "flips_explained": examine and all(f["err_one_sided"] <= 1e-5 for f in flips),
                    "rule": "every band g_u0 above 1e-5 equals an fp64 one-sided derivative at u0 +- d within 1e-5"}
            a, r = a[reg], r[reg]
        err[k] = float((a - r).abs().max() / den)
    err32 = {}
    for k in ("loss", "prediction", "xhat", "g_W_inp", "g_b_inp", "g_W_out", "g_u0"):
        r = ref[k].reshape(-1)
        a32 = ref32[k].reshape(-1).double()
        if k == "g_u0":
            a32, r = a32[reg], r[reg]
        err32[k] = float((a32 - r).abs().max() / ref[k].abs().max().clamp_min(1e-300))
    for p in ctrl.parameters():
        p.grad = None
    grads = ("g_u0", "g_W_inp", "g_b_inp", "g_W_out")
    return {"grad_max_rel_err": max(err[k] for k in grads), "torch_fp32_err": err32,
            "out_max_rel_err": max(err[k] for k in ("loss", "prediction", "xhat")),
            "per_tensor": err, "batch": B, "g_u0_kink_band": band,
            "compared": "loss/prediction/xhat and the parameter gradients over every trajectory; g_u0 outside the band",
            "oracle": "oracle/rollout_torch.py fp64 on the GPU, chunked over trajectories (checker only)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=65536, help="trajectories per GPU")
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--hidden", type=int, default=50)
    ap.add_argument("--cpu-budget", type=float, default=24.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--grad-check", choices=("full", "off"), default="full",
                    help="full: grad max-rel-err of the benchmarked batch vs the fp64 torch restatement (after timing)")
    ap.add_argument("--precision", choices=("fp32", "f16"), default="fp32",
                    help="fp32: reference-accurate (default, config 2); f16: gate products in f16 in both passes, fp32 "
                         "accumulate (config 3)")
    ap.add_argument("--graphed", action="store_true",
                    help="time the step as NeuralNetwork.captured_step replays it (one HIP graph per step; the "
                         "launch-bound small batches, e.g. the reference's B = 15); 1 GPU")
    ap.add_argument("--small-limit", type=int, default=None,
                    help="MPCLoss(small_batch_limit=...): B at or below it runs the small-batch kernels (0 = never; "
                         "default: the library's, 8192)")
    ap.add_argument("--wide-keep-budget", default=None,
                    help="H > 52: bytes of kept windows the workspace may hold (MPCLoss(wide_keep_budget=...)), in GiB, or "
                         "'max' = the device's free memory less 8 GiB. The library default keeps what fits in half the "
                         "free memory (within 40%% of HBM); a job that owns the GPU opts in to more: fewer windows "
                         "recomputed in the backward")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal of the N > 1 path on a 1-GPU box: every rank on cuda:0, gloo process group "
                         "(launcher, barriers, grad all-reduce, max-over-ranks timing); not a scaling number")
    args = ap.parse_args()

    # --gpus N without a launcher: start N ranks (torchrun) as a child BEFORE anything touches the GPU
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(fca.launch.spawn_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:]))
    rank, local, world = fca.launch.rank_env()
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.graphed and world > 1:
        sys.exit("bench.py: --graphed times the 1-GPU captured step")
    dev = torch.device("cuda", 0 if args.share_gpu else local)
    torch.cuda.set_device(dev)            # before the process group: RCCL binds each rank to its own GPU
    # the process group's timeout bounds every wait, including the other ranks' final barrier while rank 0 runs
    # its post-timing grad check (GRAD_CHECK_BUDGET_S, far inside it)
    pg_timeout = datetime.timedelta(minutes=30)
    if world > 1:
        if args.share_gpu:
            dist.init_process_group("gloo", timeout=pg_timeout)
        else:
            dist.init_process_group("nccl", device_id=dev, timeout=pg_timeout)
        world = dist.get_world_size()
    B, N, H = args.batch, args.horizon, args.hidden
    keep_budget = None
    if args.wide_keep_budget is not None:
        if args.wide_keep_budget == "max":
            free, _ = torch.cuda.mem_get_info(dev)
            keep_budget = max(0, free - (8 << 30))
        else:
            keep_budget = int(float(args.wide_keep_budget) * (1 << 30))

    sim, ctrl = load_weights(dev, H)
    if world > 1:
        fca.distributed.broadcast_params(ctrl)
    opt = torch.optim.AdamW(ctrl.parameters(), lr=1e-4)     # UL/Main.py:195
    # this loss's own kernel options (include/fcr.h fcr_options; None = the library's defaults)
    loss_fn = fca.MPCLoss(prediction_horizon=N, alpha=ALPHA, precision=args.precision,
                          small_batch_limit=args.small_limit, wide_keep_budget=keep_budget)
    sync = fca.distributed.GradAllReduce() if world > 1 else None
    X, S = synth_batch(B, dev, 1000 + rank)
    stream = torch.cuda.current_stream(dev)      # the stream the C ABI launches on
    marks = []

    def step(ev=None):
        opt.zero_grad()
        out = ctrl(X)
        if ev is not None:
            ev[0].record(stream)
        loss, feats = loss_fn(sim, ctrl, X, out, S, dev)
        if ev is not None:
            ev[1].record(stream)
        loss.backward()
        if ev is not None:
            ev[2].record(stream)
        if sync is not None:
            sync(ctrl, B, B * world, loss)
            if ev is not None:
                # after the all-reduce has been joined into the launching stream (RCCL: the collective's stream
                # is waited on by this one before dist.all_reduce returns; gloo: host-side, so the event also
                # carries the host round trip): ev[2] -> ev[3] is the step's exchange as the stream sees it
                ev[3].record(stream)
        opt.step()
        return loss

    captured = None
    if args.graphed:
        # the product's captured step (graphed.CapturedStep): warm-up steps, capture, then one replay per step
        captured = fca.NeuralNetwork.captured_step(sim, ctrl, loss_fn, opt, dev)
        for _ in range(max(args.warmup, 3)):
            captured(X, S)
    else:
        for _ in range(args.warmup):
            step()
    torch.cuda.synchronize()
    call = loss_fn.last_call   # what the warm-up steps ran: kernel families, workspace, kept windows (H > 52)
    small = call is not None and call.forward == "small"

    # timed region: K steps; HIP events on the launching stream bracket the fused forward and backward of
    # EVERY timed step (the per-kernel times come from the same steps as ms_per_step)
    marks = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        if captured is not None:
            loss = captured(X, S)[0]
        else:
            loss = step(marks[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt_local = dt
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = 1000.0 * dt / args.steps
    value = world * B * N / (dt / args.steps)
    if captured is not None:
        # graph replays carry no events between kernels: time the same kernels in a few eager steps after
        marks = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(5)]
        for k in range(len(marks)):
            step(marks[k])
        torch.cuda.synchronize()
    fwd_ms = [e[0].elapsed_time(e[1]) for e in marks]
    bwd_ms = [e[1].elapsed_time(e[2]) for e in marks]
    ar_ms = [e[2].elapsed_time(e[3]) for e in marks] if sync is not None else []
    per_rank = None
    if world > 1:
        # every rank's own means and step clock at rank 0: how far the ranks spread, and how much of the step the
        # all-reduce is (Functions.py:1463 is the shard point; the exchange is the one grad all-reduce, :658)
        mine = {"rank": rank, "device": str(dev), "fwd_ms": float(np.mean(fwd_ms)), "bwd_ms": float(np.mean(bwd_ms)),
                "allreduce_ms": float(np.mean(ar_ms)), "allreduce_max_ms": float(np.max(ar_ms)),
                "step_ms": 1000.0 * dt_local / args.steps}
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)

    if rank == 0:
        f_ms, b_ms = float(np.mean(fwd_ms)), float(np.mean(bwd_ms))
        fl = flops_per_rollout_step(H)
        dom = ("bwd", b_ms) if b_ms >= f_ms else ("fwd", f_ms)
        narrow = H <= 52
        wide_label = {   # H > 52 (fcr_wgemm.h / fcr_wbwd.h; H padded to whole 64-unit blocks)
            "fwd": "wide_cell_fwd_kernel (hand-written split-f16 GEMM + cell update)",
            "bwd": "backward pass: recompute wide_cell_fwd_kernel (windows not kept) + wide_bwd_fused_kernel (dgates on "
                   "producer waves, split-f16 [input grad | dh] product on consumer waves)"}
        kernel = (f"fcr_s{dom[0]}_kernel" if small else f"fcr_{dom[0]}_kernel") if narrow else wide_label[dom[0]]
        achieved = B * N * fl[dom[0]] / (dom[1] * 1e-3) / 1e12
        hbm_roof = HBM_PEAK_GBS * 1e9 / hbm_bytes_per_rollout_step(N)
        default_cfg = (B, N, H, args.precision) == (65536, 10, 50, "fp32")
        c5_cfg = (B, N, H, args.precision) == (65536, 25, 256, "fp32")
        c3_cfg = (B, N, H) == (262144, 10, 50)   # config 3 in either precision: its own PMC summary
        traffic, traffic_src = (pmc_traffic(f"fcr_{dom[0]}_kernel") if default_cfg else
                                pmc_traffic(f"fcr_{dom[0]}_kernel", f"_c3{args.precision}") if c3_cfg else
                                pmc_traffic("bwd_pass", "_c5") if c5_cfg and dom[0] == "bwd" else (None, None))
        # ceiling of the arithmetic as executed: an fp32-accurate product is three f16 MFMA products
        # (hi.hi + hi.lo + lo.hi, fcr_f16.h), so the fp32-equivalent ceiling is the f16 peak / 3;
        # in the reduced-precision pass one f16 product each
        f16_pass = args.precision == "f16"
        peak = F16_PEAK_TFLOPS if f16_pass else F16_PEAK_TFLOPS / 3
        roof = {"bound": "mfma", "kernel": kernel, "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                "frac": achieved / peak, "traffic": traffic,
                "traffic_unit": "bytes/launch" if narrow else "bytes per backward pass (all its dispatches)",
                "traffic_source": traffic_src,
                "achieved_def": f"algorithmic {fl[dom[0]]} FLOP per rollout-step x B*N / mean HIP-event time of the "
                                f"{dom[0]} pass over the timed steps",
                "peak_def": ("f16 dense MFMA peak (one f16 product per algorithmic product)" if f16_pass else
                             "f16 dense MFMA peak / 3: the ceiling of fp32-accurate products built from three f16 "
                             "MFMA products"),
                "fp32_peak_frac": achieved / FP32_PEAK_TFLOPS}
        if narrow and args.precision == "fp32":
            ex = executed_mfma_flop(dom[0], B, N) / (dom[1] * 1e-3) / 1e12
            roof["executed"] = {"instr": "v_mfma_f32_16x16x32_f16", "achieved": ex, "peak": F16_PEAK_TFLOPS,
                                "unit": "TFLOP/s", "frac": ex / F16_PEAK_TFLOPS,
                                "def": "MFMA FLOP issued (split products, padding, backward recompute) / time"}
        prec_label = {"fp32": "fp32", "f16": "f16 fwd+bwd"}[args.precision]
        line = {
            "metric": "rollout-steps/s (batch x horizon), fwd+bwd+AdamW step",
            "value": value, "unit": "rollout-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": {"fp32": "f32", "f16": "f16"}[args.precision],
            "data": "synthetic (SURVEY §8d distribution); reference-trained LSTM/controller weights",
            "config": {"workload": f"unsupervised-MPC rollout train step, B={B}/GPU, N={N}, H={H}, 3-layer LSTM, "
                                   f"ctrl 3-50-1, {prec_label}" + (", HIP-graph replay" if captured is not None else ""),
                       "batch_per_gpu": B, "global_batch": B * world,
                       "horizon": N, "hidden": H, "parallelism": f"dp{world}", "world_size": world,
                       "kernels": {"forward": call.forward, "backward": call.backward} if call else None,
                       **({"wide_keep_budget_gib": round(keep_budget / 2**30, 1) if keep_budget is not None
                           else "library default (half the free memory at first sizing, <= 40% of HBM)",
                           "workspace_gib": round(call.workspace_bytes / 2**30, 1),
                           "kept_windows": call.kept_windows}
                          if H > 52 and call is not None else {}),
                       **({"rehearsal": "--share-gpu: every rank on cuda:0 over gloo (path check, not a scaling "
                                        "number)"} if args.share_gpu else {})},
            "roofline": roof,
            "kernels_ms": {"fwd": f_ms, "bwd": b_ms,
                           **({"allreduce": float(np.mean(ar_ms)), "allreduce_max": float(np.max(ar_ms))}
                              if ar_ms else {}),
                           "source": ("HIP events on the launching stream, 5 eager steps after the graphed timed region"
                                      if captured is not None else
                                      "HIP events on the launching stream, every timed step")},
            **({"ranks": {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                          "step_ms_spread": max(r["step_ms"] for r in per_rank) - min(r["step_ms"] for r in per_rank),
                          "per_rank": per_rank}} if per_rank else {}),
            # the design's own HBM traffic (activation records and hand-off slabs, PMC-measured) against
            # 8 TB/s: how close the dominant kernel runs to the bandwidth its data movement needs
            "hbm_traffic_frac": (traffic / (dom[1] * 1e-3) / (HBM_PEAK_GBS * 1e9)) if traffic else None,
            "hbm_roofline_frac": value / world / hbm_roof,
            "loss": float(loss.item()),
        }
        if args.grad_check != "off":
            if keep_budget is not None:
                torch.cuda.empty_cache()   # the kept windows' workspace back to the device for the checker's chunks
            t_gc = time.perf_counter()
            gc = grad_check(sim, ctrl, X, S, N, dev, args.precision)
            gc["seconds"] = round(time.perf_counter() - t_gc, 2)
            gc["rank"] = rank
            if gc["seconds"] > GRAD_CHECK_BUDGET_S:
                print(f"bench.py: grad check took {gc['seconds']} s (budget {GRAD_CHECK_BUDGET_S} s)", file=sys.stderr)
            line["grad_max_rel_err"] = gc.pop("grad_max_rel_err")
            line["out_max_rel_err"] = gc.pop("out_max_rel_err")
            line["grad_check"] = gc
        if not args.no_cpu_baseline and world == 1:
            # the line's own workload at H > 52 (config 5); the H <= 52 lines share config 2's (per rollout-step)
            line["cpu_baseline"] = cpu_baseline(args.cpu_budget, N=N if H > 52 else 10, H=H if H > 52 else 50)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
