// fcr_window.h — device-resident window gather for the training/validation loaders.
//
// Reference: SequenceDataset.__getitem__ (Functions.py:109-132) over the per-trajectory datasets that
// Data.get_individual_dataset builds (Functions.py:479-516) and Main.py:275-279 concatenates
// (torch ConcatDataset): global sample g -> trajectory k = g / T, local row i = g % T, and
//   x = X[i], y = Y[min(i + 1, T - 1)], z[j] = Z[max(i - L + 1 + j, 0)]   (j = 0..L-1)
// all rows relative to trajectory k (the left padding repeats the trajectory's first row; windows never
// cross trajectories). The reference builds each sample in Python per item; here one launch gathers a
// whole batch from the concatenated tables in HBM.
//
// Layout: one lane per output float, samples contiguous: lane e of sample b writes x (nx floats), then
// y (ny), then z (L·nz, row-major) — stores are fully coalesced; the reads are short contiguous rows.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fcr {
namespace window {

constexpr int kWinBlock = 256;

struct WinArgs {
    const float *X, *Y, *Z;
    long long rows;
    int traj_len, lookback, nx, ny, nz;
    int B;
    const long long *idx;
    float *x, *y, *z;
    int *bad;
};

__global__ __launch_bounds__(kWinBlock) void window_gather_kernel(WinArgs a) {
    const int per = a.nx + a.ny + a.lookback * a.nz;
    const long long e = (long long)blockIdx.x * kWinBlock + threadIdx.x;
    if (e >= (long long)a.B * per) return;
    const int b = (int)(e / per);
    int k = (int)(e - (long long)b * per);
    const long long g = a.idx[b];
    const bool ok = g >= 0 && g < a.rows;
    if (!ok && k == 0) atomicAdd(a.bad, 1);
    const long long base = ok ? g - g % a.traj_len : 0;   // trajectory's first row
    const int i = ok ? (int)(g - base) : 0;
    if (k < a.nx) {
        a.x[(long long)b * a.nx + k] = ok ? a.X[(base + i) * a.nx + k] : 0.0f;
        return;
    }
    k -= a.nx;
    if (k < a.ny) {
        const int r = i + 1 < a.traj_len ? i + 1 : a.traj_len - 1;
        a.y[(long long)b * a.ny + k] = ok ? a.Y[(base + r) * a.ny + k] : 0.0f;
        return;
    }
    k -= a.ny;
    const int j = k / a.nz, f = k - j * a.nz;
    const int r = i - a.lookback + 1 + j;
    a.z[(long long)b * a.lookback * a.nz + k] = ok ? a.Z[(base + (r > 0 ? r : 0)) * a.nz + f] : 0.0f;
}

}  // namespace window
}  // namespace fcr
