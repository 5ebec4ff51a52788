"""forging-control_amd — MI355X-native (gfx950) unsupervised-MPC rollout engine.

Drop-in for the hot path of marcowus/forging-control: ``MPCLoss`` (the batched closed-loop rollout of
the FNN controller through the 3-layer LSTM plant surrogate, Functions.py:1336-1472) and its
backward, as hand-written HIP kernels behind the C ABI in include/fcr.h.
"""
from . import _native, closed_loop, data, distributed, graphed, inference, launch, plant, rollout, surrogate
from .functions import FNNModel, LSTMModel, MPCLoss, NeuralNetwork
from .inference import controller_step, simulate_step, simulator_make_step
from .plant import ForgingRK4, forging_rk4
from .data import DeviceLoader, SequenceWindows
from .closed_loop import ClosedLoop
from .graphed import CapturedStep

__all__ = ["FNNModel", "LSTMModel", "MPCLoss", "NeuralNetwork", "rollout", "distributed", "inference",
           "simulate_step", "controller_step", "simulator_make_step", "plant", "ForgingRK4", "forging_rk4",
           "data", "SequenceWindows", "DeviceLoader", "surrogate", "closed_loop", "ClosedLoop", "graphed",
           "CapturedStep", "launch", "_native"]
