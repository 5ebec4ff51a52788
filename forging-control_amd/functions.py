"""Host-side mirror of the reference's hot-path interface (Unsupervised Learning/Functions.py).

Same class names, constructor/forward signatures, parameter names (so reference ``state_dict``s load
unchanged) and return conventions as the reference. On a ROCm device the rollout inside :class:`MPCLoss`
runs on the gfx950 kernels through :mod:`.rollout` (and raises if libfcr.so is missing: no fallback
there); on the CPU — the reference's ``device = cpu`` branch (UL/Main.py:38) — it runs the reference's
own op sequence on the caller's modules, as :class:`LSTMModel` / :class:`FNNModel` already do off-device.

* :class:`FNNModel`     <- Functions.py:215-289
* :class:`LSTMModel`    <- Functions.py:295-379
* :class:`MPCLoss`      <- Functions.py:1336-1472 (the hot path, now HIP)
* :class:`NeuralNetwork` train_model / validate_model / train_loop <- Functions.py:594-717, 825-923
"""
from __future__ import annotations

import logging
import time

import torch
from torch import nn

from .rollout import rollout

logger = logging.getLogger("forging_control_amd")


class FNNModel(nn.Module):
    """Controller: Linear(in->hidden)+act, (width-1) x [Linear(hidden->hidden)+act], Linear(hidden->out,
    no bias), Hardtanh. Xavier-normal weights, zero biases (Functions.py:239-259)."""

    def __init__(self, input_dim: int, hidden_dim: int, output_dim: int, width_dim: int,
                 activation_fn=nn.ReLU, bias=True):
        super().__init__()
        self.width_dim = width_dim
        self.activation = activation_fn()
        self.constraint = nn.Hardtanh()
        self.fc_inp = nn.Linear(input_dim, hidden_dim, bias=bias)
        self.fc_int = nn.Linear(hidden_dim, hidden_dim, bias=bias)
        self.fc_out = nn.Linear(hidden_dim, output_dim, bias=False)
        for layer in (self.fc_inp, self.fc_int, self.fc_out):
            nn.init.xavier_normal_(layer.weight)
        for layer in (self.fc_inp, self.fc_int):
            if layer.bias is not None:
                nn.init.zeros_(layer.bias)

    def forward(self, x):
        """Functions.py:275-289. The reference's shape (3 -> hidden -> 1, width 1, ReLU) on a ROCm
        device runs the HIP kernels of :mod:`.controller`; other shapes are this module's torch layers."""
        from .controller import fnn_apply, hip_shape_ok
        if hip_shape_ok(self, x):
            return fnn_apply(self, x)
        y = self.activation(self.fc_inp(x))
        for _ in range(self.width_dim - 1):
            y = self.activation(self.fc_int(y))
        return self.constraint(self.fc_out(y))


class LSTMModel(nn.Module):
    """Plant surrogate: stacked ``nn.LSTM`` (batch-first, no bias by default) from a zero state, then a
    linear readout of the last step (Functions.py:317-379)."""

    def __init__(self, input_dim: int, hidden_dim: int, output_dim: int, layer_dim: int, bias=False,
                 device: torch.device = "cpu"):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.layer_dim = layer_dim
        self.lstm = nn.LSTM(input_dim, hidden_dim, layer_dim, batch_first=True, bias=bias)
        self.fc = nn.Linear(hidden_dim, output_dim)

    def initialize_hidden_states(self, batch_size: int, device: torch.device):
        shape = (self.layer_dim, batch_size, self.hidden_dim)
        return (torch.zeros(shape, device=device).requires_grad_(),
                torch.zeros(shape, device=device).requires_grad_())

    def forward(self, x: torch.Tensor, device: torch.device):
        """fc(h_9 of the top layer) from a zero state (Functions.py:353-379). The reference's shape —
        LSTM(5, H, 3) without bias on (B, 10, 5) windows, on a ROCm device — runs the gfx950 path
        (surrogate.py: fcr_lstm_forward, and fcr_lstm_backward under autograd). Anything else — above all
        the closed-loop harness's ``model(X_new, "cpu")`` on a model moved to the CPU (Functions.py:999,
        UL/Main.py:347-348) — is this module's own ``nn.LSTM`` + ``fc``, exactly the reference's forward."""
        from .surrogate import hip_shape_ok, lstm_apply
        if hip_shape_ok(self, x):
            return lstm_apply(self, x)
        h0, c0 = self.initialize_hidden_states(x.shape[0], x.device)
        out, _ = self.lstm(x, (h0.detach(), c0.detach()))
        return self.fc(out[:, -1, :])


def _controller_params(controller):
    if not isinstance(controller, FNNModel) and not all(hasattr(controller, a) for a in ("fc_inp", "fc_out")):
        raise TypeError("MPCLoss: controller must be an FNNModel (fc_inp / fc_out)")
    if getattr(controller, "width_dim", 1) != 1:
        raise NotImplementedError("MPCLoss rollout kernel is built for width_dim=1 (UL/Main.py:183)")
    if not isinstance(getattr(controller, "activation", nn.ReLU()), nn.ReLU):
        raise NotImplementedError("MPCLoss rollout kernel is built for the ReLU controller (UL/Main.py:188)")
    if controller.fc_inp.bias is None:
        raise NotImplementedError("MPCLoss rollout kernel expects fc_inp with bias (UL/Main.py:188)")
    return controller.fc_inp.weight, controller.fc_inp.bias, controller.fc_out.weight


def _simulator_params(simulator):
    lstm = simulator.lstm
    if lstm.bias:
        raise NotImplementedError("MPCLoss rollout kernel is built for the bias-free LSTM (Functions.py:317)")
    if lstm.num_layers != 3 or lstm.input_size != 5 or simulator.fc.out_features != 4:
        raise NotImplementedError("MPCLoss rollout kernel is built for LSTM(5, H, 3) -> Linear(H, 4)")
    w_ih = [getattr(lstm, f"weight_ih_l{k}") for k in range(3)]
    w_hh = [getattr(lstm, f"weight_hh_l{k}") for k in range(3)]
    return w_ih, w_hh, simulator.fc.weight, simulator.fc.bias


class MPCLoss(nn.Module):
    """Drop-in for the reference MPCLoss (Functions.py:1336-1472): the N-step closed-loop rollout of the
    controller through the LSTM surrogate and its quadratic speed-tracking cost, fused on gfx950 (CPU
    tensors: the reference's own op sequence, :meth:`_forward_host`).

    ``forward`` returns ``(loss, {'loss', 'command', 'error', 'prediction'})`` with the reference's
    shapes. ``enable_noise`` draws ``randn_like(x0) * 0.01`` per horizon step from the device's default
    generator in the reference's order (Functions.py:1401, 1439); a pre-drawn ``noise`` (B, N, 4) can be
    passed instead. After each call ``self.last_trajectory`` holds the (B, N, 4) LSTM predictions.

    Kernel options of THIS loss (include/fcr.h fcr_options, carried from each forward to its backward; None inherits
    the process-wide default): ``small_batch_limit`` — B at or below it runs the small-batch kernels (0 = never);
    ``wide_keep_budget`` — H > 52, bytes of kept windows the workspace may add ("auto": the library's policy).
    ``self.last_call`` (a :class:`~.rollout.CallInfo`) reports the kernel families the last call's passes launched
    and its workspace.
    """

    def __init__(self, prediction_horizon=10, alpha=0.1, precision="fp32", small_batch_limit=None,
                 wide_keep_budget=None):
        super().__init__()
        self.N = prediction_horizon
        self.alpha = alpha
        self.precision = precision     # "fp32" (reference-accurate) or "f16" (config 3, include/fcr.h)
        self.small_batch_limit = small_batch_limit
        self.wide_keep_budget = wide_keep_budget
        self.activation = nn.ReLU()
        self.last_trajectory = None
        self.last_call = None

    def forward(self, simulator: nn.Module, controller: nn.Module, input_controller: torch.Tensor,
                output_controller: torch.Tensor, states: torch.Tensor, device: torch.device,
                enable_noise=False, noise: torch.Tensor | None = None):
        X = input_controller
        dev = torch.device(device)
        if dev.type != X.device.type or (dev.index is not None and dev.index != X.device.index):
            raise RuntimeError(f"MPCLoss: inputs are on {X.device}, device argument is {device}")
        B = X.shape[0]
        if X.device.type == "cpu":
            return self._forward_host(simulator, controller, X, output_controller, states, device, enable_noise, noise)
        if enable_noise and noise is None:
            noise = torch.stack([torch.randn(B, 4, device=X.device) * 0.01 for _ in range(self.N)], dim=1)
        elif not enable_noise:
            noise = None
        from . import _native
        from .rollout import CallInfo
        self.last_call = CallInfo(_native.make_options(self.small_batch_limit, self.wide_keep_budget))
        loss, cost, command, error, prediction, xhat = rollout(
            X, output_controller, states, _controller_params(controller), _simulator_params(simulator),
            self.N, self.alpha, noise, self.precision, self.last_call)
        self.last_trajectory = xhat
        return loss, {"loss": cost, "command": command, "error": error, "prediction": prediction}

    def _forward_host(self, simulator, controller, X, u0, states, device, enable_noise, noise):
        """The rollout where the reference runs it without a GPU (``device = cpu``, UL/Main.py:38): its op
        sequence (Functions.py:1386-1472) on the caller's own modules — ``simulator(window, device)`` and
        ``controller(x)`` are LSTMModel's / FNNModel's torch layers off-device — under autograd, so
        ``loss.backward()`` reaches the controller parameters and ``output_controller`` as the reference's
        does (the frozen LSTM's weight gradients included). Noise: ``randn_like(x̂) * 0.01`` drawn after every
        surrogate call in the reference's order (:1400-1402, :1438-1440), or the given (B, N, 4) ``noise``."""
        N, alpha, relu = self.N, self.alpha, self.activation
        B = X.shape[0]

        def perturb(xh, j):
            if noise is not None and enable_noise:
                return xh + noise[:, j]
            if enable_noise:
                return xh + torch.randn_like(xh) * 0.01
            return xh

        def constraint(xh):                                                       # Functions.py:1411, 1449
            return relu(-xh[:, 1]) + relu(-xh[:, 2]) + relu(xh[:, 1] - 2.122366) + relu(xh[:, 2] - 1.036233)

        ref = X[:, -1]                                                            # :1392
        window = states.clone()                                                   # :1395-1396
        window[:, -1, -1] = u0.reshape(B)
        xh = perturb(simulator(window, device), 0)                                # :1399-1402
        cmd = [alpha * torch.square(window[:, -2, -1] - window[:, -1, -1])]       # :1405
        err = [torch.square(xh[:, 0] - ref)]                                      # :1408
        tot = [err[0] + cmd[0] + constraint(xh)]                                  # :1414
        u_next = u0.reshape(B, 1)
        preds, traj = [u_next], [xh]
        for j in range(N - 1):                                                    # :1421
            u_prev = u_next
            u_next = controller(torch.stack((xh[:, 0], xh[:, 3], ref), dim=1))    # :1424-1430
            window = torch.cat((window[:, 1:10, :], torch.cat((xh, u_next), dim=1).unsqueeze(1)), dim=1)   # :1433-1434
            xh = perturb(simulator(window, device), j + 1)                        # :1437-1440
            err.append(torch.square(xh[:, 0] - ref))                              # :1443
            cmd.append(alpha * torch.square(u_prev.reshape(B) - u_next.reshape(B)))   # :1446
            tot.append(err[-1] + cmd[-1] + constraint(xh))                        # :1449-1452
            preds.append(u_next)
            traj.append(xh)
        cost = torch.stack(tot).sum(dim=0) / N                                    # :1458-1460
        command = torch.stack(cmd).sum(dim=0) / N
        error = torch.stack(err).sum(dim=0) / N
        self.last_trajectory = torch.stack(traj, dim=1).detach()
        return cost.mean(), {"loss": cost, "command": command, "error": error,    # :1463-1472
                             "prediction": torch.cat(preds, dim=1).flatten()}


class NeuralNetwork:
    """Training driver with the reference's call surface (Functions.py:594-923)."""

    @staticmethod
    def captured_step(simulator, model, loss_function, optimizer, device, enable_noise=False, grad_sync=None,
                      warmup=2):
        """The body of :meth:`train_model`'s batch loop as a :class:`~.graphed.CapturedStep` (one HIP graph
        replay per batch; pass it as ``train_model(..., step=...)``, reusable across epochs)."""
        from .graphed import CapturedStep

        def body(X, z):
            output = model(X)
            loss, f = loss_function(simulator, model, X, output, z, device, enable_noise)
            loss.backward()
            return (loss.detach(), f["loss"], f["command"], f["error"], f["prediction"])

        sync = (lambda X, z: grad_sync(model, X.shape[0])) if grad_sync is not None else None
        return CapturedStep(model.parameters(), optimizer, body, sync, warmup)

    @staticmethod
    def train_model(data_loader, simulator, model, loss_function, optimizer, device, enable_noise=False,
                    grad_sync=None, step=None):
        """One epoch (Functions.py:594-676). ``grad_sync`` (optional) is called as ``grad_sync(model, B_local)``
        between backward and the optimizer step — the data-parallel hook (:class:`.distributed.GradAllReduce`
        weights each rank's gradient by its batch size, so uneven shards give the global-mean gradient). ``step`` (optional, from
        :meth:`captured_step`) replays each batch's step from a HIP graph; the epoch's loss is then summed
        on the device and read once, not per batch."""
        model.train()
        if step is not None:
            return NeuralNetwork._train_model_captured(data_loader, step, device)
        total = 0.0
        feats = {"loss": [], "command": [], "error": [], "prediction": []}
        n_batches = 0
        for X, _, z in data_loader:
            X, z = X.to(device), z.to(device)
            optimizer.zero_grad()
            if X.shape[0] == 0:
                # an empty shard (more ranks than trajectories in a short last batch): no rollout, but the
                # rank still joins the all-reduce with b_local = 0 and steps with everyone's gradient
                if grad_sync is not None:
                    grad_sync(model, 0)
                    optimizer.step()
                continue
            output = model(X)
            loss, f = loss_function(simulator, model, X, output, z, device, enable_noise)
            for k in feats:
                feats[k].append(f[k])
            loss.backward()
            if grad_sync is not None:
                grad_sync(model, X.shape[0])   # this rank's batch: the hook weights it into the global mean
            optimizer.step()
            total += loss.item()
            n_batches += 1
        feats = {k: torch.cat(v, dim=0) if v else torch.empty(0, device=device) for k, v in feats.items()}
        return total / max(n_batches, 1), feats

    @staticmethod
    def _train_model_captured(data_loader, step, device):
        keys = ("loss", "command", "error", "prediction")
        feats = {k: [] for k in keys}
        total = None
        n_batches = 0
        for X, _, z in data_loader:
            X, z = X.to(device), z.to(device)
            if X.shape[0] == 0:   # an empty shard: join the all-reduce and step, as the eager loop does
                step.skip_empty(X, z)
                continue
            loss, *f = step(X, z)
            total = loss.clone() if total is None else total + loss
            for k, v in zip(keys, f):
                feats[k].append(v.clone())
            n_batches += 1
        avg = float(total.item()) / n_batches if n_batches else 0.0
        return avg, {k: torch.cat(v, dim=0) if v else torch.empty(0, device=device) for k, v in feats.items()}

    @staticmethod
    def validate_model(data_loader, model, loss_function, device):
        """Controller-only validation loss (Functions.py:679-717)."""
        model.eval()
        total = 0.0
        n = 0
        with torch.no_grad():
            for X, y, _ in data_loader:
                X, y = X.to(device), y.to(device)
                total += loss_function(model(X), y).item()
                n += 1
        return total / n if n else 0.0

    @staticmethod
    def predict(data_loader, model):
        """Controller predictions over a loader (Functions.py:720-748): ``model(X)`` per batch, evaluation
        mode, no gradients, concatenated along the batch. The batches go to the device the model lives on
        (the reference leaves that to the loader); on a ROCm device that is the HIP controller kernel."""
        model.eval()
        dev = next(model.parameters()).device
        preds = []
        with torch.no_grad():
            for X, _, _ in data_loader:
                preds.append(model(X.to(dev)))
        return torch.cat(preds, dim=0)

    @staticmethod
    def simulator_make_step(X, model, scalers, noise):
        """Functions.py:969-1011: the surrogate's unscaled one-step prediction for the closed-loop harness
        (see :func:`.inference.simulator_make_step`; runs where the model is)."""
        from .inference import simulator_make_step
        return simulator_make_step(X, model, scalers, noise)

    @staticmethod
    def train_loop(controller, simulator, train_loader, val_loader, loss_function, optimizer, n_epochs,
                   device, enable_noise=False, grad_sync=None, graphed=False):
        """Epoch loop (Functions.py:825-923); returns (controller, train losses, val losses, seconds,
        stacked loss features). ``graphed=True`` replays every batch's step from one HIP graph
        (:meth:`captured_step`) — for the launch-bound small batches the reference trains with."""
        NeuralNetwork.validate_model(val_loader, controller, nn.MSELoss(), device)
        step = (NeuralNetwork.captured_step(simulator, controller, loss_function, optimizer, device, enable_noise,
                                            grad_sync) if graphed else None)
        t_losses, v_losses = [], []
        stacked = {"loss": [], "command": [], "error": [], "prediction": []}
        t0 = time.time()
        for epoch in range(n_epochs):
            tl, f = NeuralNetwork.train_model(train_loader, simulator, controller, loss_function, optimizer,
                                              device, enable_noise, grad_sync, step)
            vl = NeuralNetwork.validate_model(val_loader, controller, nn.MSELoss(), device)
            if n_epochs >= 10 and epoch % (n_epochs // 10) == 0 or epoch == n_epochs - 1:
                logger.info("[%.1f%%] Training loss: %.4f,  Validation loss: %.4f",
                            100.0 * epoch / n_epochs, tl, vl)
            t_losses.append(tl)
            v_losses.append(vl)
            for k in stacked:
                stacked[k].append(f[k].detach())
        elapsed = time.time() - t0
        stacked = {k: torch.stack(v, dim=0) for k, v in stacked.items()}
        return controller, t_losses, v_losses, elapsed, stacked
