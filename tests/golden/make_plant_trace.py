"""Extract the reference's closed-loop press traces as a fixture (data only, no code).

Source: /root/reference/Unsupervised Learning/results/{MPC,Unsupervised}_dataframe.txt — the rows the
harness writes (UL/Main.py:908-935): time, ref, y, y_dot, p1, p2, z, u at TS = 1 ms, printed %.6f.
Output: tests/golden/plant_trace.npz with one (T, 8) float64 array per file. Run in the container that
holds /root/reference; the GPU box only reads the .npz.
"""
import os

import numpy as np

SRC = "/root/reference/Unsupervised Learning/results"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "plant_trace.npz")

if __name__ == "__main__":
    arrays = {}
    for name in ("MPC", "Unsupervised"):
        path = os.path.join(SRC, f"{name}_dataframe.txt")
        with open(path) as f:
            header = f.readline().split()
        assert header == ["time", "ref", "y", "y_dot", "p1", "p2", "z", "u"], header
        arrays[name.lower()] = np.loadtxt(path, skiprows=1)
    np.savez_compressed(OUT, columns=np.array(header), **arrays)
    print(OUT, {k: v.shape for k, v in arrays.items()})
