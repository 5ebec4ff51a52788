// fcr_closed_loop.h — the NN controller driving the press, all T steps of B trajectories in one launch
// (SURVEY.md §8(f) ranks 1 + 2 together: the closed-loop evaluation the plant row exists for).
//
// Reference: NeuralNetwork.loop (Functions.py:1075-1240) without feasibility recovery, per step t:
//   X = [y_dot, z, ref_t]; X_new = scalers['input'].transform(X) with the last column replaced by
//   scalers['y_dot'].transform(ref_t) (NN_make_step, Functions.py:1594-1598); u = scalers['output']
//   .inverse_transform(FNN(float32(X_new))) (:1601-1604); x_{t+1} = plant(x_t, u) (:1178-1179; here the
//   reference's own RK4 integrator F of Ruge_Kuta, Functions.py:1743-1781, in place of do-mpc's CVODES).
// The scalers are MaxAbsScalers (UL/Main.py:237-256): transform = x / scale, inverse = x · scale.
//
// One lane owns one trajectory: fp64 state in VGPRs for all T steps, the 3->H->1 controller in fp32 as
// torch evaluates it (weights in LDS, one FMA chain per hidden unit), the plant in fp64. HBM sees the
// reference (8 B) in and u (8 B) + the state (40 B) out per step.
#pragma once
#include <hip/hip_runtime.h>

#include "fcr_plant.h"

namespace fcr {
namespace closed_loop {

constexpr int kClBlock = 256;
constexpr int kClMaxHidden = 256;

struct ClArgs {
    int B, T, substeps, hidden;
    double dt;
    const double *x0, *ref;
    const float *w_inp, *b_inp, *w_out;
    double in_scale0, in_scale1, ref_scale, out_scale;
    double *x, *u;
};

template <bool SMOOTH>
__global__ __launch_bounds__(kClBlock) void closed_loop_kernel(ClArgs a) {
    __shared__ float w[kClMaxHidden * 5];        // [j] = (w_inp[j][0..2], b_inp[j], w_out[j])
    for (int i = threadIdx.x; i < a.hidden; i += kClBlock) {
        w[i * 5 + 0] = a.w_inp[i * 3 + 0];
        w[i * 5 + 1] = a.w_inp[i * 3 + 1];
        w[i * 5 + 2] = a.w_inp[i * 3 + 2];
        w[i * 5 + 3] = a.b_inp[i];
        w[i * 5 + 4] = a.w_out[i];
    }
    __syncthreads();
    const int b = blockIdx.x * kClBlock + threadIdx.x;
    if (b >= a.B) return;
    double x[5];
    double *o = a.x + (size_t)b * (a.T + 1) * 5;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        x[i] = a.x0[(size_t)b * 5 + i];
        o[i] = x[i];
    }
    const double *rb = a.ref + (size_t)b * a.T;
    double *ub = a.u + (size_t)b * a.T;
    for (int t = 0; t < a.T; ++t) {
        // NN_make_step: scaled input in fp64, then float32 for the torch model (Functions.py:1594-1601)
        const float s0 = (float)(x[1] / a.in_scale0), s1 = (float)(x[4] / a.in_scale1), s2 = (float)(rb[t] / a.ref_scale);
        float v = 0.0f;
        for (int j = 0; j < a.hidden; ++j) {   // fc_inp + ReLU, fc_out (no bias) (Functions.py:275-287)
            const float *wj = w + j * 5;
            float z = fmaf(wj[2], s2, fmaf(wj[1], s1, fmaf(wj[0], s0, wj[3])));
            z = z > 0.0f ? z : 0.0f;
            v = fmaf(wj[4], z, v);
        }
        v = fminf(fmaxf(v, -1.0f), 1.0f);                 // Hardtanh
        const double u = (double)(v * (float)a.out_scale); // inverse_transform on the float32 output
        ub[t] = u;
        plant::rk4_step<SMOOTH>(x, u, a.dt, a.substeps);
        o += 5;
#pragma unroll
        for (int i = 0; i < 5; ++i) o[i] = x[i];
    }
}

}  // namespace closed_loop
}  // namespace fcr
