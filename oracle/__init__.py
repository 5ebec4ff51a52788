"""Oracle: CPU restatements of the reference (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and the CPU-baseline legs of ``bench.py`` and
``scripts/bench_*.py`` may import this package, and only as the checker / CPU baseline; nothing in
``forging-control_amd/`` imports it.

| module | restates | parity pin |
|---|---|---|
| ``rollout_np`` (fp64 NumPy, hand-written reverse pass) | MPCLoss forward + backward | unpinned by reference fixtures (none exist; its Python may not run here) — cross-checked against ``rollout_torch`` to ~1e-15 |
| ``rollout_torch`` (stock torch ops, reference op order) | the same, plus the rollout's CPU baseline | second restatement for the above |
| ``plant_np`` | forging_model / template_model + Ruge_Kuta | pinned on the reference's closed-loop traces (``tests/golden/plant_trace.npz``) |
| ``closed_loop_np`` | NeuralNetwork.loop without feasibility recovery | composed of ``plant_np`` and the FNN |
| ``windows_ref`` | SequenceDataset.__getitem__ + ConcatDataset | line-by-line restatement of the indexing |
| ``surrogate_torch`` | Model_NN train_model body (MSE + AdamW) | autograd, checked by finite differences |

See DESIGN.md §3 and §7.
"""
